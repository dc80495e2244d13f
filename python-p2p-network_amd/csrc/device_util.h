// Device helpers shared by the relay kernels (relay_kernels.hip, relay_grouped.hip): wave
// reductions / scans (DPP), scalar-cached loads, non-temporal row stores, bitmap tests, and
// the host-side grid sizing of the grid-stride task kernels.  Internal; not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "internal.h"
#include "philox.h"

namespace p2pg {
namespace {

constexpr int WPB = 4;  // waves per block (256 threads)
// Sparse-round kernels scan this many task words per wave pass, one per lane
#ifndef P2PG_SCAN_W
#define P2PG_SCAN_W 4
#endif
constexpr int SCAN_W = P2PG_SCAN_W;
constexpr int GRID_MAX = 2048;

__device__ __forceinline__ bool bit_test(const uint32_t* bm, int64_t v) {
  return (bm[v >> 5] >> (v & 31)) & 1u;
}

__device__ __forceinline__ uint64_t full_mask(int w, int W, int M) {
  if (w < W - 1 || (M & 63) == 0) return ~0ull;
  return (1ull << (M & 63)) - 1ull;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// Wave-wide 32-bit reductions through DPP row shifts and row broadcasts (gfx9 family):
// four row_shr steps reduce each 16-lane row into its lane 15, row_bcast:15 / row_bcast:31
// fold the rows into lane 63, which is then read as a scalar.
template <bool MAX>
__device__ __forceinline__ uint32_t wave_reduce_u32(uint32_t x) {
  auto op = [](uint32_t a, uint32_t b) { return MAX ? (a > b ? a : b) : a + b; };
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// Inclusive prefix sum over the wave (the same DPP steps as wave_reduce_u32<false>).
__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}

__device__ __forceinline__ void flush_stats(unsigned long long* stats, const uint64_t* c,
                                            int lane) {
  unsigned long long* shard = stats + (blockIdx.x & (STAT_SHARDS - 1)) * STAT_N;
#pragma unroll
  for (int i = 0; i < STAT_N; ++i) {
    const uint64_t s = wave_sum(c[i]);
    if (lane == 0 && s) atomicAdd(shard + i, (unsigned long long)s);
  }
}

// Load through the constant address space: a wave-uniform address then becomes a scalar
// load (s_load, counted on lgkmcnt) instead of a vector load whose vmcnt wait would also wait
// for every row store the wave still has in flight.  Only for data no kernel writes.
template <class T>
__device__ __forceinline__ T ldc(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
}

// Per-connection E stores of the gossip dense rounds are non-temporal: the planes are re-read
// a round later, far beyond L2 / MALL reach, and nt stores retire sooner -- which matters
// because a wave's next gather wait (vmcnt, in order) also waits for its in-flight stores
// (c4 A/B: fused rounds 267.9 -> 258.7 ms per step).  P2PG_NT_STORE=0 restores plain stores.
// P2PG_NT_ROWS / P2PG_NT_LOADS extend nt to the fused kernel's seen / frontier row stores and
// to its E gathers (read once per receiver): together another 260.6 -> 258.7 ms (3 interleaved
// pairs).
#ifndef P2PG_NT_STORE
#define P2PG_NT_STORE 1
#endif
#ifndef P2PG_NT_ROWS
#define P2PG_NT_ROWS 1
#endif
#ifndef P2PG_NT_LOADS
#define P2PG_NT_LOADS 1
#endif
#ifndef P2PG_NT_ISSUE
#define P2PG_NT_ISSUE 0
#endif
// streamed-once loads of the fused kernel's row stage (seen word, neighbour ids, receiver slots);
// nt here measured ±0 (3 interleaved c4 pairs), so off by default
template <class T>
__device__ __forceinline__ T ld_once(const T* p) {
#if P2PG_NT_ISSUE
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
__device__ __forceinline__ void st_row(uint64_t* p, uint64_t x) {
#if P2PG_NT_STORE
  __builtin_nontemporal_store(x, p);
#else
  *p = x;
#endif
}
#ifndef P2PG_NT_PULL
#define P2PG_NT_PULL 1  // c4 update kernel 13.3 -> 12.7 ms per step; c3 flood pull unchanged
#endif
// seen / frontier / push-row stores of the pull and update kernels, non-temporal too
__device__ __forceinline__ void st_prow(uint64_t* p, uint64_t x) {
#if P2PG_NT_PULL
  __builtin_nontemporal_store(x, p);
#else
  *p = x;
#endif
}
__device__ __forceinline__ void st_frow(uint64_t* p, uint64_t x) {
#if P2PG_NT_ROWS
  __builtin_nontemporal_store(x, p);
#else
  *p = x;
#endif
}

// Row r of a [rows][W] plane for a per-lane row id.  Row ids (peers, and E slots: rev[] holds
// them as uint32) and W fit 32 bits, so the offset is one 32 x 32 -> 64 multiply-add per lane;
// an int64 product takes two v_mad_u64_u32 and moves (the grouped kernel's gathers: W = 8 share
// 67.8 -> 65.4 ms, profiles/r06/ab_grouped_addr.txt).
template <class T>
__device__ __forceinline__ T* at_row(T* plane, uint64_t r, int W) {
  // byte offset r x (W x 8): the row stride in bytes is kernel-constant, so the per-lane form is
  // one v_mad_u64_u32 with the plane as its addend and the scalar form has no 64-bit shift
  using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
  const uint32_t stride = (uint32_t)W * (uint32_t)sizeof(T);
  return reinterpret_cast<T*>(reinterpret_cast<B*>(plane) + (uint64_t)(uint32_t)r * stride);
}

// Global peer id of a local vertex (partitioned runs keep ghosts in global-id order; the
// Philox keys of churn and gossip are global ids so partitioning cannot change results).
__device__ __forceinline__ uint32_t gidx(const DevGraph& g, int64_t x) {
  return g.gid ? (uint32_t)g.gid[x] : (uint32_t)x;
}

// Same for a wave-uniform vertex: a scalar load (see ldc), no vmcnt wait.
__device__ __forceinline__ uint32_t gidx_s(const DevGraph& g, int64_t x) {
  const int64_t xu = __builtin_amdgcn_readfirstlane((int)x);
  return g.gid ? (uint32_t)ldc(g.gid + xu) : (uint32_t)xu;
}

// The activity word of a task at the end of a (phase of a) round: a phase-1 pass adds its
// peers' bits to those of phase 0; a whole-round or phase-0 pass writes the word.
__device__ __forceinline__ void put_active(uint32_t* A, int64_t task, uint32_t aw, const RoundParams& p) {
  if (p.phase == 1)
    A[task] |= aw;
  else
    A[task] = aw;
}

// wave index inside the block, forced into an SGPR so task indices stay scalar
__device__ __forceinline__ int wave_in_block() {
  return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

__device__ __forceinline__ int64_t readlane64(int64_t x, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Lane-varying register read (ds_bpermute).  Every call site runs with the whole wave active:
// a disabled source lane would not deliver its value.
__device__ __forceinline__ uint32_t bperm(int src_lane, uint32_t x) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)x);
}

__device__ __forceinline__ uint64_t bperm64(int src_lane, uint64_t x) {
  return ((uint64_t)bperm(src_lane, (uint32_t)(x >> 32)) << 32) | bperm(src_lane, (uint32_t)x);
}

// Inclusive running maximum over the wave (the DPP steps of wave_scan_u32; 0 is the identity).
__device__ __forceinline__ uint32_t wave_scan_max_u32(uint32_t x) {
  auto mx = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
  x = mx(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
  x = mx(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
  x = mx(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
  x = mx(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
  x = mx(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
  x = mx(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
  return x;
}

// Position of the n-th (0-based) set bit of x; n < popcount(x).
__device__ __forceinline__ uint32_t select_bit32(uint32_t x, uint32_t n) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t s = 16; s; s >>= 1) {
    const uint32_t c = (uint32_t)__popc(x & ((1u << s) - 1u));
    const bool up = n >= c;
    n = up ? n - c : n;
    x = up ? x >> s : x;
    pos = up ? pos + s : pos;
  }
  return pos;
}

__device__ __forceinline__ uint32_t select_bit64(uint64_t x, uint32_t n) {
  const uint32_t lo = (uint32_t)x;
  const uint32_t cl = (uint32_t)__popc(lo);
  const bool up = n >= cl;
  return (up ? 32u : 0u) + select_bit32(up ? (uint32_t)(x >> 32) : lo, up ? n - cl : n);
}

// Word-major list of the set bits of every lane's 64-bit word f (the gossip pick lists, DESIGN.md
// 4a): the r-th set bit b of lane l's word becomes entry (tag | b) at position li0 + r, li0 = the
// lane's exclusive prefix of popcounts minus the entries of earlier passes (wrapping: positions
// below the pass are never written); positions >= cap belong to a later pass.  Entries that are
// not written go to lst[dummy] (one address for all lanes: an LDS broadcast, no bank conflict).
// Two entries per lane per trip -- the r-th bit of each 32-bit half, the high half's entries
// following the low half's -- and a wave-uniform trip count (the largest half popcount), so the
// loop has no divergence and no exec-mask bookkeeping (the per-bit loop it replaces ran the low
// and the high half one after the other, ~17 instructions per bit, with lanes dropping out).
__device__ __forceinline__ void list_bits(uint16_t* lst, uint32_t dummy, uint64_t f, uint32_t tag,
                                          uint32_t li0, uint32_t cap) {
  uint32_t lo = (uint32_t)f, hi = (uint32_t)(f >> 32);
  const uint32_t pl = (uint32_t)__popc(lo), ph = (uint32_t)__popc(hi);
  const uint32_t trips = wave_reduce_u32<true>(pl > ph ? pl : ph);
  uint32_t al = li0, ah = li0 + pl;
  const uint32_t th = tag | 32u;
  for (uint32_t t = 0; t < trips; ++t) {
    // (bit 31 forced on: a defined ctz when the half is empty -- that entry goes to the dummy)
    const uint32_t bl = (uint32_t)__builtin_ctz(lo | 0x80000000u);
    const uint32_t bh = (uint32_t)__builtin_ctz(hi | 0x80000000u);
    lst[(t < pl && al < cap) ? al : dummy] = (uint16_t)(tag | bl);
    lst[(t < ph && ah < cap) ? ah : dummy] = (uint16_t)(th | bh);
    lo &= lo - 1u;
    hi &= hi - 1u;
    ++al;
    ++ah;
  }
}

// Orders this wave's LDS writes before its later LDS reads by other lanes.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Blocks of `kernel` (256 threads) that fit on the whole device at once: a persistent grid of
// exactly this size has no second, partial wave of blocks (no tail).
template <class F>
int resident_blocks(F kernel) {
  static const void* key[32];
  static int val[32];
  static int n = 0;
  for (int i = 0; i < n; ++i)
    if (key[i] == (const void*)kernel) return val[i];
  int nb = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, 256, 0) != hipSuccess || nb < 1) nb = 1;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  const int r = nb * cus;
  if (n < 32) {
    key[n] = (const void*)kernel;
    val[n] = r;
    ++n;
  }
  return r;
}

int grid_tasks_uncapped(int64_t ntasks) {
  const int64_t b = (ntasks + WPB - 1) / WPB;
  return (int)(b < 1 ? 1 : (b > 0x7FFFFFFF ? 0x7FFFFFFF : b));
}

// Grid of a grid-stride task kernel: one 4-wave block per 4 tasks, at most grid_max() blocks
// (P2PG_GRID_MAX, default GRID_MAX).  Many more blocks than fit at once: a block that drew
// cheap tasks is replaced by the next one, which evens out the per-wave cost.
int grid_max() {
  static const int g = [] {
    const char* e = std::getenv("P2PG_GRID_MAX");
    const int v = e ? std::atoi(e) : GRID_MAX;
    return v > 0 ? v : GRID_MAX;
  }();
  return g;
}

int grid_tasks(int64_t ntasks) {
  int64_t b = (ntasks + WPB - 1) / WPB;
  const int64_t cap = grid_max();
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

// Grid for the per-peer pull kernels, whose task cost is very uneven (power-law degrees,
// receipts per peer): P2PG_FUSED_GRID (default 32) x the blocks resident at once, so that
// blocks finishing early are replaced (measured on config 4: 2x -> 300 ms, 8x -> 267 ms,
// 32x -> 260 ms for the fused rounds).
// The fused / grouped kernels keep their per-wave round totals in 32 bits.  A 32-peer task adds
// at most 32 peers x 4096 messages x fanout 16 = 2^21 to any of them (relays; hubs, deg > HUB_T,
// never go through these kernels, so wedges <= 32 x 64 words x 512 = 2^20), so a wave may take
// at most 2^10 tasks (2^10 x 2^21 = 2^31 < 2^32, strictly): the grid is never smaller than that
// bound asks, whatever P2PG_FUSED_GRID, the device size or V (config 4: ~2.4 tasks per wave).
constexpr int64_t TASKS_PER_WAVE_MAX = 1024;
static_assert(TASKS_PER_WAVE_MAX * (int64_t{32} * 4096 * 16) < (int64_t{1} << 32),
              "per-wave 32-bit round totals could wrap");

template <class F>
int balanced_grid(F kernel, int64_t ntasks) {
  static const int gmul = [] {
    const char* e = std::getenv("P2PG_FUSED_GRID");
    const int v = e ? std::atoi(e) : 32;
    return v > 0 ? v : 32;
  }();
  const int64_t full = (int64_t)grid_tasks_uncapped(ntasks);
  const int64_t floor32 = (ntasks + TASKS_PER_WAVE_MAX * WPB - 1) / (TASKS_PER_WAVE_MAX * WPB);
  return (int)std::min<int64_t>(full, std::max<int64_t>((int64_t)gmul * resident_blocks(kernel), floor32));
}


}  // namespace
}  // namespace p2pg
