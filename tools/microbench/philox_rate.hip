// Microbenchmark: Philox4x32-10 throughput on gfx950 (how much VALU the gossip picks cost).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
struct u4 { uint32_t x, y, z, w; };
__device__ __forceinline__ u4 philox_a(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    u4 n = { (uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0 };
    c = n; k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c;
}
__device__ __forceinline__ u4 philox_b(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t h0 = __umulhi(0xD2511F53u, c.x), l0 = 0xD2511F53u * c.x;
    uint32_t h1 = __umulhi(0xCD9E8D57u, c.z), l1 = 0xCD9E8D57u * c.z;
    u4 n = { h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0 };
    c = n; k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c;
}
// v_bitop3_b32 (gfx950): the two XORs of each output word as one 3-input op (LUT 0x96)
__device__ __forceinline__ u4 philox_c(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    u4 n = { (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
             (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0 };
    c = n; k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c;
}
template <int V>
__global__ void run(uint64_t n, uint32_t* out) {
  extern __shared__ uint32_t pad[];
  if (n == 0) pad[threadIdx.x] = 0;  // dynamic LDS only limits occupancy
  uint32_t acc = 0;
  uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = gridDim.x * (uint64_t)blockDim.x;
  for (uint64_t i = t; i < n; i += nt) {
    u4 c = {(uint32_t)i, (uint32_t)(i >> 32), 7u, 0x475350u};
    u4 r = V == 0 ? philox_a(c, 1u, 2u) : (V == 1 ? philox_b(c, 1u, 2u) : philox_c(c, 1u, 2u));
    acc += r.x ^ r.y ^ r.z ^ r.w;
  }
  if (acc == 0x12345u) out[0] = acc;
}
int main() {
  uint32_t* out; CK(hipMalloc(&out, 64));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  uint64_t n = 1ull << 32;
  for (int lds : {0, 20 * 1024, 36 * 1024, 64 * 1024}) {
    for (int v = 0; v < 3; v += 2) {
      printf("dynamic LDS %d B/block: ", lds);
      auto L = [&] {
        if (v == 0) run<0><<<256 * 16, 256, lds>>>(n, out);
        else run<2><<<256 * 16, 256, lds>>>(n, out);
      };
      L(); CK(hipDeviceSynchronize());
      CK(hipEventRecord(a)); L(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      printf("variant %d: %.3f ms for 2^32 philox calls -> %.1f G calls/s\n", v, ms, n / (ms * 1e6));
    }
  }
  return 0;
}
