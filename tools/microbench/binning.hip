// Microbenchmark for the sparse-round push design (not part of the product): random 8 B
// atomicOr into planes of several sizes (does a smaller, cache-resident footprint help?),
// against binning the same pushes -- 16 B records, a counting sort by target range (per-block
// LDS histograms, no per-record global atomics), and an LDS-resident apply per bucket.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

// n pushes: push i -> word (target(i), w(i)) of a [V][W] plane, mask 1 << (i & 63)
__global__ void atomics(uint64_t* plane, uint32_t V, int W, uint64_t n) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = gridDim.x * (uint64_t)blockDim.x;
  for (uint64_t i = t; i < n; i += nt) {
    const uint32_t h = hash32((uint32_t)i);
    const uint64_t tg = h % V, w = hash32(h) % (uint32_t)W;
    atomicOr((unsigned long long*)&plane[tg * W + w], 1ull << (i & 63));
  }
}

// the same pushes written as records (key = word index, mask)
__global__ void records(uint64_t* key, uint64_t* val, uint32_t V, int W, uint64_t n) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = gridDim.x * (uint64_t)blockDim.x;
  for (uint64_t i = t; i < n; i += nt) {
    const uint32_t h = hash32((uint32_t)i);
    const uint64_t tg = h % V, w = hash32(h) % (uint32_t)W;
    key[i] = tg * W + w;
    val[i] = 1ull << (i & 63);
  }
}

constexpr int NB = 4096;     // buckets per pass
constexpr int CHUNK = 65536;  // records per block
__global__ __launch_bounds__(256) void hist(const uint64_t* key, uint64_t n, int shift, uint32_t* h) {
  __shared__ uint32_t l[NB];
  for (int i = threadIdx.x; i < NB; i += 256) l[i] = 0;
  __syncthreads();
  const uint64_t b0 = (uint64_t)blockIdx.x * CHUNK;
  for (uint64_t i = b0 + threadIdx.x; i < n && i < b0 + CHUNK; i += 256) atomicAdd(&l[(key[i] >> shift) & (NB - 1)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < NB; i += 256) h[(uint64_t)i * gridDim.x + blockIdx.x] = l[i];
}
__global__ __launch_bounds__(256) void scatter(const uint64_t* key, const uint64_t* val, uint64_t n, int shift,
                                               const uint32_t* off, uint64_t* okey, uint64_t* oval) {
  __shared__ uint32_t c[NB];
  for (int i = threadIdx.x; i < NB; i += 256) c[i] = off[(uint64_t)i * gridDim.x + blockIdx.x];
  __syncthreads();
  const uint64_t b0 = (uint64_t)blockIdx.x * CHUNK;
  for (uint64_t i = b0 + threadIdx.x; i < n && i < b0 + CHUNK; i += 256) {
    const uint64_t k = key[i];
    const uint32_t p = atomicAdd(&c[(k >> shift) & (NB - 1)], 1u);
    okey[p] = k;
    oval[p] = val[i];
  }
}
// apply: bucket b = records of targets [b << tb, (b+1) << tb), ORed in LDS, rows written out
__global__ __launch_bounds__(256) void apply(const uint64_t* key, const uint64_t* val, const uint32_t* start,
                                             int W, int tb, uint64_t* plane) {
  extern __shared__ uint64_t tbl[];
  const int rows = 1 << tb;
  for (int i = threadIdx.x; i < rows * W; i += 256) tbl[i] = 0;
  __syncthreads();
  const uint32_t b = blockIdx.x;
  for (uint32_t i = start[b] + threadIdx.x; i < start[b + 1]; i += 256) {
    const uint64_t k = key[i] - ((uint64_t)b << tb) * W;
    if (k < (uint64_t)rows * W) atomicOr((unsigned long long*)&tbl[k], (unsigned long long)val[i]);
  }
  __syncthreads();
  uint64_t* dst = plane + ((uint64_t)b << tb) * W;
  for (int i = threadIdx.x; i < rows * W; i += 256)
    if (tbl[i]) dst[i] |= tbl[i];
}

int main() {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float ms;
  auto timeit = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a)); for (int k = 0; k < 3; ++k) launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b)); ms /= 3;
    printf("%-52s %8.3f ms\n", name, ms);
    return ms;
  };
  const uint64_t n = 80000000ull;  // ~ a c4 round-9 / W = 8 round-11 sparse push
  uint64_t* plane;
  CK(hipMalloc(&plane, 10000000ull * 64 * 8));
  for (auto vw : {std::pair<uint32_t, int>{10000000u, 64}, {10000000u, 8}, {1000000u, 8}, {125000u, 8}}) {
    char nm[96];
    snprintf(nm, 96, "atomicOr 8B, %u x %d plane (%.0f MB)", vw.first, vw.second, vw.first * vw.second * 8.0 / 1e6);
    timeit(nm, [&] { atomics<<<4096, 256>>>(plane, vw.first, vw.second, n); });
  }
  uint64_t *k0, *v0, *k1, *v1;
  CK(hipMalloc(&k0, n * 8)); CK(hipMalloc(&v0, n * 8)); CK(hipMalloc(&k1, n * 8)); CK(hipMalloc(&v1, n * 8));
  const int nblk = (int)((n + CHUNK - 1) / CHUNK);
  uint32_t *h, *off;
  CK(hipMalloc(&h, sizeof(uint32_t) * NB * nblk + 64)); CK(hipMalloc(&off, sizeof(uint32_t) * NB * nblk + 64));
  void* tmp = nullptr;
  size_t tmpb = 0;
  hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, h, off, NB * nblk);
  CK(hipMalloc(&tmp, tmpb));
  for (int W : {64, 8}) {
    const uint32_t V = 10000000u;
    const int tb = W == 64 ? 5 : 8;  // rows per apply bucket: 16 KB of LDS
    printf("-- W = %d, %llu pushes\n", W, (unsigned long long)n);
    timeit("records (16 B each, sequential)", [&] { records<<<4096, 256>>>(k0, v0, V, W, n); });
    // bucket id = target >> tb = key >> (tb + log2 W); two passes of 12 bits cover V >> tb < 2^24
    const int lw = W == 64 ? 6 : 3;
    float tot = 0;
    for (int pass = 0; pass < 2; ++pass) {
      const int shift = lw + tb + 12 * pass;
      const uint64_t* ki = pass ? k1 : k0;
      const uint64_t* vi = pass ? v1 : v0;
      uint64_t* ko = pass ? k0 : k1;
      uint64_t* vo = pass ? v0 : v1;
      char nm[96];
      snprintf(nm, 96, "counting sort pass %d (hist + scan + scatter)", pass);
      tot += timeit(nm, [&] {
        hist<<<nblk, 256>>>(ki, n, shift, h);
        hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, h, off, NB * nblk);
        scatter<<<nblk, 256>>>(ki, vi, n, shift, off, ko, vo);
      });
    }
    printf("%-52s %8.3f ms\n", "  two passes", tot);
    // the library's stable radix sort on the bucket bits, for comparison (and a correct grouping)
    {
      int nbits = 1;
      while ((1u << nbits) < (V >> tb)) ++nbits;
      void* t2 = nullptr;
      size_t t2b = 0;
      hipcub::DeviceRadixSort::SortPairs(t2, t2b, k0, k1, v0, v1, (int)n, lw + tb, lw + tb + nbits);
      CK(hipMalloc(&t2, t2b));
      timeit("records again", [&] { records<<<4096, 256>>>(k0, v0, V, W, n); });
      timeit("hipcub DeviceRadixSort::SortPairs on bucket bits", [&] {
        hipcub::DeviceRadixSort::SortPairs(t2, t2b, k0, k1, v0, v1, (int)n, lw + tb, lw + tb + nbits);
      });
      CK(hipMemcpy(k0, k1, n * 8, hipMemcpyDeviceToDevice));
      CK(hipMemcpy(v0, v1, n * 8, hipMemcpyDeviceToDevice));
      CK(hipFree(t2));
    }
    // bucket starts from the sorted keys (host-side here: the product would fold it into a scan)
    const uint32_t nbk = V >> tb;
    std::vector<uint64_t> hk(n);
    CK(hipMemcpy(hk.data(), k0, n * 8, hipMemcpyDeviceToHost));
    std::vector<uint32_t> st(nbk + 1, 0);
    for (uint64_t i = 0; i < n; ++i) st[(hk[i] >> lw >> tb) + 1]++;
    bool sorted = true;
    for (uint64_t i = 1; i < n && sorted; ++i) sorted = (hk[i] >> lw >> tb) >= (hk[i - 1] >> lw >> tb);
    for (uint32_t i = 0; i < nbk; ++i) st[i + 1] += st[i];
    uint32_t* dst;
    CK(hipMalloc(&dst, sizeof(uint32_t) * (nbk + 1)));
    CK(hipMemcpy(dst, st.data(), sizeof(uint32_t) * (nbk + 1), hipMemcpyHostToDevice));
    printf("  sorted by bucket: %s\n", sorted ? "yes" : "NO");
    timeit("apply (LDS OR per bucket, rows ORed into the plane)", [&] {
      apply<<<nbk, 256, (size_t)(1 << tb) * W * 8>>>(k0, v0, dst, W, tb, plane);
    });
    CK(hipFree(dst));
  }
  return 0;
}
