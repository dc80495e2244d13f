// Philox4x32-10 counter-based RNG, shared by host (generators, sources) and device (gossip
// picks, churn mask) so that every random decision is a pure function of its counter.
//
// Constants: Salmon et al., "Parallel random numbers: as easy as 1, 2, 3" (SC'11) /
// Random123; same values as /opt/rocm/include/rocrand/rocrand_philox4x32_10.h:62-65.
// Known-answer vectors (Random123 kat_vectors) are pinned in tests/test_philox.py.
//
// Counter layouts used by the engine:
//   sources : key = (seed_lo, seed_hi ^ TAG_SRC), ctr = (msg_global, 0, 0, 0)
//   gossip  : key = (seed_lo, seed_hi),           ctr = (round, peer, msg_global, TAG_GSP | blk<<24)
//   churn   : key = (seed_lo, seed_hi),           ctr = (round, min(a,b), max(a,b), TAG_CHN)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define P2PG_HD __host__ __device__ __forceinline__
#else
#define P2PG_HD static inline
#endif

namespace p2pg {

constexpr uint32_t PHILOX_M0 = 0xD2511F53u;
constexpr uint32_t PHILOX_M1 = 0xCD9E8D57u;
constexpr uint32_t PHILOX_W0 = 0x9E3779B9u;
constexpr uint32_t PHILOX_W1 = 0xBB67AE85u;

constexpr uint32_t TAG_SRC = 0x00535243u;  // 'SRC'
constexpr uint32_t TAG_GSP = 0x00475350u;  // 'GSP'
constexpr uint32_t TAG_CHN = 0x0043484Eu;  // 'CHN'
constexpr uint32_t TAG_RRG = 0x00525247u;  // 'RRG' random-regular generator
constexpr uint32_t TAG_GNP = 0x00474E50u;  // 'GNP'
constexpr uint32_t TAG_BAG = 0x00424147u;  // 'BAG' Barabasi-Albert generator
constexpr uint32_t TAG_WSG = 0x00575347u;  // 'WSG' Watts-Strogatz generator

struct u32x4 { uint32_t x, y, z, w; };

P2PG_HD u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  // 32x32->64 products as one 64-bit multiply: lowers to v_mad_u64_u32 on gfx950, which the
  // microbenchmark (tools/microbench/philox_rate.hip) measured 1.3x faster than mul_hi+mul_lo.
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)PHILOX_M0 * c.x;
    const uint64_t p1 = (uint64_t)PHILOX_M1 * c.z;
    u32x4 n;
#if defined(__HIP_DEVICE_COMPILE__)
    // gfx950 v_bitop3_b32 (LUT 0x96 = a ^ b ^ c): one VALU op per output word instead of two
    n.x = (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96);
    n.z = (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96);
#else
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
#endif
    n.y = (uint32_t)p1;
    n.w = (uint32_t)p0;
    c = n;
    k0 += PHILOX_W0;
    k1 += PHILOX_W1;
  }
  return c;
}

// Lemire multiply-high reduction of a 32-bit draw onto [0, n).
P2PG_HD uint32_t lemire32(uint32_t x, uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(x, n);  // one v_mul_hi_u32, and a 32-bit value for the Floyd compares
#else
  return (uint32_t)(((uint64_t)x * (uint64_t)n) >> 32);
#endif
}

P2PG_HD uint32_t word_of(const u32x4& r, int i) {
  return i == 0 ? r.x : (i == 1 ? r.y : (i == 2 ? r.z : r.w));
}

// Push-gossip target choice: k distinct indices into the sender's ascending
// adjacency list of length n, by Floyd's algorithm; draw i uses word (i % 4) of Philox block
// (i / 4).  Requires n > k (callers send to every neighbour when n <= k).  Writes the k
// picks to out[0..k) in draw order.  K_MAX bounds the storage of the caller.
P2PG_HD void gossip_picks(uint32_t round, uint32_t peer, uint32_t msg, uint32_t n, int k,
                          uint32_t seed_lo, uint32_t seed_hi, uint32_t* out) {
  u32x4 r = {0, 0, 0, 0};
  for (int i = 0; i < k; ++i) {
    if ((i & 3) == 0) {
      u32x4 c = {round, peer, msg, TAG_GSP | ((uint32_t)(i >> 2) << 24)};
      r = philox4x32_10(c, seed_lo, seed_hi);
    }
    const uint32_t jmax = n - (uint32_t)k + (uint32_t)i;  // Floyd: candidate range [0, jmax]
    uint32_t t = lemire32(word_of(r, i & 3), jmax + 1u);
    bool dup = false;
    for (int q = 0; q < i; ++q) dup |= (out[q] == t);
    out[i] = dup ? jmax : t;
  }
}

// Same draws with k fixed at compile time, so out[] stays in registers on the device (a
// runtime-indexed private array would live in scratch memory).
template <int K>
P2PG_HD void gossip_picks_t(uint32_t round, uint32_t peer, uint32_t msg, uint32_t n,
                            uint32_t seed_lo, uint32_t seed_hi, uint32_t (&out)[K]) {
  u32x4 r = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < K; ++i) {
    if ((i & 3) == 0) {
      u32x4 c = {round, peer, msg, TAG_GSP | ((uint32_t)(i >> 2) << 24)};
      r = philox4x32_10(c, seed_lo, seed_hi);
    }
    const uint32_t jmax = n - (uint32_t)K + (uint32_t)i;
    const uint32_t t = lemire32(word_of(r, i & 3), jmax + 1u);
    bool dup = false;
#pragma unroll
    for (int q = 0; q < i; ++q) dup |= (out[q] == t);
    out[i] = dup ? jmax : t;
  }
}

// The gossip draws of one source (round, peer fixed) for many messages, k <= 4 (one Philox block
// per message).  In the counter (round, peer, msg, TAG_GSP) only msg varies, so the first two
// Philox rounds have wave-uniform parts: they are folded into per-source constants once
// (PickKey, scalar registers on the device), and a message costs 18 multiplies and 19 XORs
// instead of 20 + 20 and the extra moves of XORs with two scalar operands.  Same outputs as
// philox4x32_10 (checked against it, tests/test_philox.py and every GPU gossip parity test).
struct PickKey {
  uint32_t a1, d2, f2, g3;  // peer ^ k0; hi(M1 z1) ^ k0'; lo(M0 round) ^ k1'; lo(M1 z1) ^ k0''
  uint32_t k0, k1;          // the key (rounds 3.. use k + i * W)
};

P2PG_HD PickKey pick_key(uint32_t round, uint32_t peer, uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)PHILOX_M0 * round;           // round 1, uniform half
  const uint32_t z1 = (uint32_t)(p0 >> 32) ^ TAG_GSP ^ k1;
  const uint32_t w1 = (uint32_t)p0;
  const uint64_t q1 = (uint64_t)PHILOX_M1 * z1;              // round 2, uniform half
  PickKey k;
  k.a1 = peer ^ k0;
  k.d2 = (uint32_t)(q1 >> 32) ^ (k0 + PHILOX_W0);
  k.f2 = w1 ^ (k1 + PHILOX_W1);
  k.g3 = (uint32_t)q1 ^ (k0 + 2u * PHILOX_W0);
  k.k0 = k0;
  k.k1 = k1;
  return k;
}

// philox4x32_10((round, peer, msg, TAG_GSP), k0, k1) for the source of pick_key
P2PG_HD u32x4 philox_pick(const PickKey& k, uint32_t msg) {
  // round 1: x = hi(M1 msg) ^ peer ^ k0, y = lo(M1 msg); z, w uniform (in d2 / f2 / g3)
  uint64_t p1 = (uint64_t)PHILOX_M1 * msg;
  const uint32_t x1 = (uint32_t)(p1 >> 32) ^ k.a1, y1 = (uint32_t)p1;
  // round 2: p0 = M0 x1 (per message), p1 = M1 z1 (uniform)
  uint64_t p0 = (uint64_t)PHILOX_M0 * x1;
  const uint32_t x2 = y1 ^ k.d2;
  const uint32_t z2 = (uint32_t)(p0 >> 32) ^ k.f2;
  const uint32_t w2 = (uint32_t)p0;
  // round 3: y2 (uniform) is in g3
  p0 = (uint64_t)PHILOX_M0 * x2;
  p1 = (uint64_t)PHILOX_M1 * z2;
  u32x4 c;
  c.x = (uint32_t)(p1 >> 32) ^ k.g3;
  c.y = (uint32_t)p1;
#if defined(__HIP_DEVICE_COMPILE__)
  c.z = (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), w2, k.k1 + 2u * PHILOX_W1, 0x96);
#else
  c.z = (uint32_t)(p0 >> 32) ^ w2 ^ (k.k1 + 2u * PHILOX_W1);
#endif
  c.w = (uint32_t)p0;
  uint32_t k0 = k.k0 + 3u * PHILOX_W0, k1 = k.k1 + 3u * PHILOX_W1;
#pragma unroll
  for (int i = 3; i < 10; ++i) {
    p0 = (uint64_t)PHILOX_M0 * c.x;
    p1 = (uint64_t)PHILOX_M1 * c.z;
    u32x4 n;
#if defined(__HIP_DEVICE_COMPILE__)
    n.x = (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96);
    n.z = (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96);
#else
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
#endif
    n.y = (uint32_t)p1;
    n.w = (uint32_t)p0;
    c = n;
    k0 += PHILOX_W0;
    k1 += PHILOX_W1;
  }
  return c;
}

// gossip_picks_t for one source's PickKey (K <= 4: one Philox block), 32-bit Floyd compares.
template <int K>
P2PG_HD void gossip_picks_k(const PickKey& key, uint32_t msg, uint32_t n, uint32_t (&out)[K]) {
  static_assert(K >= 1 && K <= 4, "one Philox block");
  const u32x4 r = philox_pick(key, msg);
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const uint32_t jmax = n - (uint32_t)K + (uint32_t)i;
    const uint32_t t = lemire32(word_of(r, i), jmax + 1u);
    bool dup = false;
#pragma unroll
    for (int q = 0; q < i; ++q) dup |= (out[q] == t);
    out[i] = dup ? jmax : t;
  }
}

// Churn: a send over undirected edge {a,b} made in round r is lost iff the
// first Philox word is below the threshold floor(p_drop * 2^32).
P2PG_HD bool churn_dropped(uint32_t round, uint32_t a, uint32_t b, uint32_t threshold,
                           uint32_t seed_lo, uint32_t seed_hi) {
  if (threshold == 0u) return false;
  const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
  u32x4 c = {round, lo, hi, TAG_CHN};
  return philox4x32_10(c, seed_lo, seed_hi).x < threshold;
}

}  // namespace p2pg
