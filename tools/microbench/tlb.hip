// Microbenchmark: random 512 B row gathers / stores vs buffer footprint (TLB reach).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
__global__ void row_read(const uint64_t* __restrict__ buf, uint64_t R, uint64_t items, uint64_t* out) {
  uint64_t acc = 0; int lane = threadIdx.x & 63;
  uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t i = wave; i < items; i += nw) { uint64_t r = ((uint64_t)hash32((uint32_t)i) * 2654435761ull + i) % R; acc |= buf[r * 64 + lane]; }
  if (acc == 0x123456789ull) out[0] = acc;
}
__global__ void row_store(uint64_t* __restrict__ buf, uint64_t R, uint64_t items) {
  int lane = threadIdx.x & 63;
  uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t i = wave; i < items; i += nw) { uint64_t r = ((uint64_t)hash32((uint32_t)i) * 2654435761ull + i) % R; buf[r * 64 + lane] = i | lane; }
}
__global__ void seq_store(uint64_t* __restrict__ buf, uint64_t R, uint64_t items) {
  int lane = threadIdx.x & 63;
  uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t i = wave; i < items; i += nw) { buf[(i % R) * 64 + lane] = i | lane; }
}
int main() {
  uint64_t* out; CK(hipMalloc(&out, 64));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const uint64_t items = 20000000ull;  // 10.24 GB of rows touched per launch
  for (double gb : {2.0, 8.0, 20.0, 41.0, 82.0}) {
    uint64_t R = (uint64_t)(gb * 1e9 / 512);
    uint64_t* buf; CK(hipMalloc(&buf, R * 512)); CK(hipMemset(buf, 0, R * 512));
    float ms;
    auto T = [&](const char* nm, auto L) {
      L(); CK(hipDeviceSynchronize());
      CK(hipEventRecord(a)); L(); L(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b)); ms /= 2;
      printf("%5.0f GB buffer  %-10s %7.3f ms  %7.1f GB/s\n", gb, nm, ms, items * 512.0 / (ms * 1e6));
    };
    T("row_read", [&] { row_read<<<2048, 256>>>(buf, R, items, out); });
    T("row_store", [&] { row_store<<<2048, 256>>>(buf, R, items); });
    T("seq_store", [&] { seq_store<<<2048, 256>>>(buf, R, items); });
    CK(hipFree(buf));
  }
  return 0;
}
