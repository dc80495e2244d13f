// Microbenchmark: 64 B rows (a W = 8 E row) -- random gathers vs random stores vs sequential,
// 8 rows per wave instruction (lane = (row g, word w)), over a 5 GB plane (config 4's E plane at
// W = 8: 80M slots x 64 B).  Also 128 B rows (W = 16) and atomics-free read+write mixes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
// RW = words per row (8: 64 B, 16: 128 B); each wave instruction covers 64 / RW rows
template <int RW>
__global__ void rnd_read(const uint64_t* __restrict__ buf, uint64_t R, uint64_t rows, uint64_t* out) {
  constexpr int G = 64 / RW;
  const int lane = threadIdx.x & 63, g = lane / RW, w = lane % RW;
  uint64_t acc = 0;
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t i = wave * G; i < rows; i += nw * G) {
    const uint64_t r = ((uint64_t)hash32((uint32_t)(i + g)) * 2654435761ull + i + g) % R;
    acc |= buf[r * RW + w];
  }
  if (acc == 0x123456789ull) out[0] = acc;
}
template <int RW>
__global__ void rnd_store(uint64_t* __restrict__ buf, uint64_t R, uint64_t rows) {
  constexpr int G = 64 / RW;
  const int lane = threadIdx.x & 63, g = lane / RW, w = lane % RW;
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t i = wave * G; i < rows; i += nw * G) {
    const uint64_t r = ((uint64_t)hash32((uint32_t)(i + g)) * 2654435761ull + i + g) % R;
    buf[r * RW + w] = i | lane;
  }
}
template <int RW>
__global__ void rnd_store_nt(uint64_t* __restrict__ buf, uint64_t R, uint64_t rows) {
  constexpr int G = 64 / RW;
  const int lane = threadIdx.x & 63, g = lane / RW, w = lane % RW;
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t i = wave * G; i < rows; i += nw * G) {
    const uint64_t r = ((uint64_t)hash32((uint32_t)(i + g)) * 2654435761ull + i + g) % R;
    __builtin_nontemporal_store(i | lane, &buf[r * RW + w]);
  }
}
template <int RW>
__global__ void seq_read(const uint64_t* __restrict__ buf, uint64_t R, uint64_t rows, uint64_t* out) {
  constexpr int G = 64 / RW;
  const int lane = threadIdx.x & 63;
  uint64_t acc = 0;
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t i = wave * G; i < rows; i += nw * G) acc |= buf[(i % R) * RW + lane];
  if (acc == 0x123456789ull) out[0] = acc;
}
int main() {
  uint64_t* out; CK(hipMalloc(&out, 64));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const uint64_t bytes = 5120000000ull;  // 5.12 GB plane
  uint64_t* buf; CK(hipMalloc(&buf, bytes)); CK(hipMemset(buf, 0, bytes));
  float ms;
  auto T = [&](const char* nm, int rw, uint64_t rows, auto L) {
    L(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a)); L(); L(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b)); ms /= 2;
    const double gb = rows * rw * 8.0 / 1e9;
    printf("%-14s row %3d B  %6.2f GB  %7.3f ms  %7.1f GB/s  %6.2f G rows/s\n", nm, rw * 8, gb, ms, gb * 1e3 / ms, rows / (ms * 1e6));
  };
  for (int grid : {2048, 8192}) {
    printf("grid %d x 256\n", grid);
    {
      const uint64_t R = bytes / 64, rows = 80000000ull;
      T("rnd_read", 8, rows, [&] { rnd_read<8><<<grid, 256>>>(buf, R, rows, out); });
      T("rnd_store", 8, rows, [&] { rnd_store<8><<<grid, 256>>>(buf, R, rows); });
      T("rnd_store_nt", 8, rows, [&] { rnd_store_nt<8><<<grid, 256>>>(buf, R, rows); });
      T("seq_read", 8, rows, [&] { seq_read<8><<<grid, 256>>>(buf, R, rows, out); });
    }
    {
      const uint64_t R = bytes / 128, rows = 40000000ull;
      T("rnd_read", 16, rows, [&] { rnd_read<16><<<grid, 256>>>(buf, R, rows, out); });
      T("rnd_store", 16, rows, [&] { rnd_store<16><<<grid, 256>>>(buf, R, rows); });
      T("rnd_store_nt", 16, rows, [&] { rnd_store_nt<16><<<grid, 256>>>(buf, R, rows); });
    }
    {
      const uint64_t R = bytes / 512, rows = 10000000ull;
      T("rnd_read", 64, rows, [&] { rnd_read<64><<<grid, 256>>>(buf, R, rows, out); });
      T("rnd_store", 64, rows, [&] { rnd_store<64><<<grid, 256>>>(buf, R, rows); });
    }
  }
  CK(hipFree(buf));
  return 0;
}
