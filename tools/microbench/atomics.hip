// Microbenchmark: which scatter/gather shapes does MI355X sustain for 64-bit bitset rows?
// Informs the relay-kernel design (DESIGN.md "design measurements"). Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
// one wave per "item"; item i touches row r(i) = hash(i) % R, lane = word
__global__ void row_read(const uint64_t* __restrict__ buf, uint64_t R, uint64_t items, uint64_t* out) {
  uint64_t acc = 0; int lane = threadIdx.x & 63;
  uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t i = wave; i < items; i += nw) { uint64_t r = hash32((uint32_t)i) % R; acc |= buf[r * 64 + lane]; }
  if (acc == 0x123456789ull) out[0] = acc;
}
__global__ void row_store(uint64_t* __restrict__ buf, uint64_t R, uint64_t items) {
  int lane = threadIdx.x & 63;
  uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t i = wave; i < items; i += nw) { uint64_t r = hash32((uint32_t)i) % R; buf[r * 64 + lane] = i | lane; }
}
__global__ void row_atomic_or(uint64_t* __restrict__ buf, uint64_t R, uint64_t items) {
  int lane = threadIdx.x & 63;
  uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * (uint64_t)blockDim.x) >> 6;
  for (uint64_t i = wave; i < items; i += nw) { uint64_t r = hash32((uint32_t)i) % R; atomicOr((unsigned long long*)&buf[r * 64 + lane], 1ull << (i & 63)); }
}
// each lane its own random row & word: 8-byte scattered atomics
__global__ void scat_atomic_or(uint64_t* __restrict__ buf, uint64_t R, uint64_t n) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = gridDim.x * (uint64_t)blockDim.x;
  for (uint64_t i = t; i < n; i += nt) { uint32_t h = hash32((uint32_t)i); uint64_t r = h % R; atomicOr((unsigned long long*)&buf[r * 64 + (hash32(h) & 63)], 1ull << (i & 63)); }
}
__global__ void scat_read(const uint64_t* __restrict__ buf, uint64_t R, uint64_t n, uint64_t* out) {
  uint64_t acc = 0;
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = gridDim.x * (uint64_t)blockDim.x;
  for (uint64_t i = t; i < n; i += nt) { uint32_t h = hash32((uint32_t)i); uint64_t r = h % R; acc |= buf[r * 64 + (hash32(h) & 63)]; }
  if (acc == 0x123456789ull) out[0] = acc;
}
// the same with the old value consumed (a returning atomic: what a push-time dedup would need)
__global__ void scat_atomic_or_ret(uint64_t* __restrict__ buf, uint64_t R, uint64_t n, uint64_t* out) {
  uint64_t acc = 0;
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = gridDim.x * (uint64_t)blockDim.x;
  for (uint64_t i = t; i < n; i += nt) { uint32_t h = hash32((uint32_t)i); uint64_t r = h % R; acc += atomicOr((unsigned long long*)&buf[r * 64 + (hash32(h) & 63)], 1ull << (i & 63)); }
  if (acc == 0x123456789ull) out[0] = acc;
}
// plain scattered 8 B stores (one lane, one random row: a lane-per-peer E-row writer)
__global__ void scat_store(uint64_t* __restrict__ buf, uint64_t R, uint64_t n) {
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = gridDim.x * (uint64_t)blockDim.x;
  for (uint64_t i = t; i < n; i += nt) { uint32_t h = hash32((uint32_t)i); uint64_t r = h % R; buf[r * 64 + (hash32(h) & 63)] = i; }
}
// sequential streaming read for calibration
__global__ void seq_read(const uint4* __restrict__ buf, uint64_t n16, uint4* out) {
  uint4 acc = {0,0,0,0};
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = gridDim.x * (uint64_t)blockDim.x;
  for (uint64_t i = t; i < n16; i += nt) { uint4 v = buf[i]; acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w; }
  if (acc.x == 0x12345678u) out[0] = acc;
}
int main() {
  const uint64_t R = 10000000ull;  // 10M rows x 512 B = 5.12 GB
  uint64_t* buf; uint64_t* out;
  CK(hipMalloc(&buf, R * 512)); CK(hipMalloc(&out, 64)); CK(hipMemset(buf, 0, R * 512));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int blocks = 256 * 16, threads = 256;
  float ms;
  auto timeit = [&](const char* name, double bytes, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a)); for (int k = 0; k < 3; ++k) launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b)); ms /= 3;
    printf("%-28s %8.3f ms  %8.1f GB/s (payload bytes)\n", name, ms, bytes / (ms * 1e6));
  };
  uint64_t items = R;  // one row-touch per row on average
  timeit("seq_read 5.12GB", R * 512.0, [&] { seq_read<<<blocks, threads>>>((const uint4*)buf, R * 32, (uint4*)out); });
  timeit("row_read 512B rows", items * 512.0, [&] { row_read<<<blocks, threads>>>(buf, R, items, out); });
  timeit("row_store 512B rows", items * 512.0, [&] { row_store<<<blocks, threads>>>(buf, R, items); });
  timeit("row_atomic_or 512B rows", items * 512.0, [&] { row_atomic_or<<<blocks, threads>>>(buf, R, items); });
  uint64_t n = 200000000ull;
  timeit("scat_read 8B", n * 8.0, [&] { scat_read<<<blocks, threads>>>(buf, R, n, out); });
  timeit("scat_atomic_or 8B", n * 8.0, [&] { scat_atomic_or<<<blocks, threads>>>(buf, R, n); });
  timeit("scat_atomic_or_ret 8B", n * 8.0, [&] { scat_atomic_or_ret<<<blocks, threads>>>(buf, R, n, out); });
  timeit("scat_store 8B", n * 8.0, [&] { scat_store<<<blocks, threads>>>(buf, R, n); });
  for (int occ : {2, 4, 8, 32}) {
    char nm[64]; snprintf(nm, 64, "row_read grid=%dx256", 256 * occ);
    timeit(nm, items * 512.0, [&] { row_read<<<256 * occ, threads>>>(buf, R, items, out); });
    snprintf(nm, 64, "row_atomic_or grid=%dx256", 256 * occ);
    timeit(nm, items * 512.0, [&] { row_atomic_or<<<256 * occ, threads>>>(buf, R, items); });
  }
  CK(hipFree(buf)); CK(hipFree(out));
  return 0;
}
