// HIP kernels (gfx950 / CDNA4) of the broadcast/relay engine.
//
// Data layout in HBM (one engine = one GPU):
//   seen, F[2], next[2] : uint64 planes [V][W], row = one peer, bit (m & 63) of word (m >> 6)
//                         = message m; W = 64 words = 512 B rows at 4096 concurrent broadcasts
//   A[2], T[2], S       : 1 bit per peer (uint32 words); A = "first receipt this round",
//                         T = "gossip pushes landed this round", S = "all messages seen"
//   rowptr int64 [V+1], colidx int32 [nnz] (ascending neighbour ids per row)
// A frontier row F[r&1][v] is only valid while A[r&1] has v's bit: rows are written whole
// (zeros included) whenever the bit is set, so nothing is ever cleared plane-wide.
//
// Reference semantics (p2pnetwork): a peer that receives a broadcast for the first time
// forwards it to every connection except the sender (Node.send_to_nodes(data,
// exclude=[sender]), node.py:106-112, one send_to_node per target, node.py:114-120) and drops
// later copies (app dedup, README.md:20).  Round-synchronous: all sends of round r-1 arrive in
// round r; the parent is the lowest-id neighbour whose copy arrived first.  Relays per first
// receipt: deg-1 (deg at the origin); gossip: min(k, deg).
//
// Wave model: one 64-lane wave per peer row, lane = word of the row, so every frontier/seen
// access is one coalesced 512 B row access (measured 5.3 TB/s for random 512 B row gathers,
// tools/microbench/atomics.hip).  Tasks = 32-peer bitmap words, grid-stride over a fixed grid
// so stats need few atomics.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "device_util.h"

// Dense pushes: the folded-round Philox of one source's draws (philox_pick); 0 = the generic
// philox4x32_10 per draw (A/B builds)
// scatter_row<.., DIRECT>: a slice with at most one new bit per word takes its picks lane = word,
// without the compacted list (P2PG_PICK_DIRECT=0: always the list; A/B).  Taken by the fused
// kernel's first-dense-round modes (push-only, update + push): c4 round 10 7.4 -> 6.9 ms; in the
// fused rounds proper the extra path cost more in the peak rounds than it saved in the light
// ones (211.2 -> 211.9 ms per step, profiles/r06/ab_pick_direct.txt)
#ifndef P2PG_PICK_DIRECT
#define P2PG_PICK_DIRECT 1
#endif
#ifndef P2PG_PICK_FOLD
#define P2PG_PICK_FOLD 1
#endif


namespace p2pg {
namespace {

// ---------------------------------------------------------------------------------------
// Round 0: origination.  Each message m sets its bit at src[m] in F[0] and seen, and the
// peer's A[0] bit (Node.send_to_nodes at the origin, node.py:106).
__global__ void k_zero_rows(uint64_t* plane, int32_t W, const int32_t* rows, int32_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * W) return;
  const int64_t r = rows[i / W];
  plane[r * W + (i % W)] = 0ull;
}

__global__ void k_seed(DevState st, const int32_t* src, int32_t M) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  const int64_t v = src[m];
  const uint64_t bit = 1ull << (m & 63);
  const int64_t o = v * st.W + (m >> 6);
  atomicOr((unsigned long long*)&st.F[0][o], (unsigned long long)bit);
  atomicOr((unsigned long long*)&st.seen[o], (unsigned long long)bit);
  atomicOr(&st.A[0][v >> 5], 1u << (v & 31));
  if (st.AW[0]) atomicOr((unsigned long long*)&st.AW[0][v], 1ull << (m >> 6));
}

// ---------------------------------------------------------------------------------------
// Pull form of a round r >= 1, shared by
//   flood  (GOSSIP = false): sources are the round-(r-1) frontier rows F[(r-1)&1][v] of the
//          active neighbours v (a flood sends the whole new set to every connection);
//   gossip (GOSSIP = true):  sources are the per-connection masks E[slot] (receiver-major:
//          slot = u's own CSR slot of the connection) that the active neighbours stored in
//          round r-1 (dense rounds, see k_gossip_scatter<STORE_E>).
// For every unsaturated peer u: OR the source rows (arrivals of round r), mask with ~seen
// (dedup), write the new frontier row and A bit.  Reads only -- no atomics (row atomics
// measured 4x slower than row reads on MI355X).  Lanes whose word is full skip their loads;
// up to 8 neighbour rows are in flight per wave.
template <bool CHURN, bool GOSSIP>
__global__ __launch_bounds__(256) void k_pull(DevGraph g, DevState st, RoundParams p) {
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int64_t V = g.V;
  const int W = st.W;
  const int cur = p.round & 1, prv = cur ^ 1;
  const uint64_t* __restrict__ Src = GOSSIP ? st.E[prv] : st.F[prv];
  uint64_t* __restrict__ Fc = st.F[cur];
  const uint32_t* __restrict__ Ap = st.A[prv];
  const int64_t ntasks = (V + 31) >> 5;
  const int nslices = (W + 63) >> 6;
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};

  for (int64_t task = (int64_t)blockIdx.x * WPB + wib; task < ntasks;
       task += (int64_t)gridDim.x * WPB) {
    const int64_t u0 = task << 5;
    const uint32_t sat0 = st.S[task];
    uint32_t sat = sat0;
    uint32_t todo = ~sat0 & phase_mask(p, task);
    if (V - u0 < 32) todo &= (1u << (V - u0)) - 1u;
    uint32_t aw = 0;
    while (todo) {
      const int b = __builtin_ctz(todo);
      todo &= todo - 1u;
      const int64_t u = u0 + b;
      const int64_t beg = g.rowptr[u], end = g.rowptr[u + 1];
      const uint64_t deg = (uint64_t)(end - beg);
      const uint64_t per_bit = GOSSIP ? (deg < (uint64_t)p.fanout ? deg : (uint64_t)p.fanout)
                                      : deg - 1;
      bool row_new = false, row_full = true;
      for (int sl = 0; sl < nslices; ++sl) {
        const int w = sl * 64 + lane;
        const bool valid = w < W;
        const uint64_t fm = valid ? full_mask(w, W, st.M) : 0ull;
        const uint64_t s = valid ? st.seen[u * W + w] : 0ull;
        const uint64_t need = fm & ~s;
        uint64_t acc = 0;
        if (__ballot(need != 0ull)) {
          for (int64_t cb = beg; cb < end; cb += 64) {
            const int64_t j = cb + lane;
            uint32_t srow = 0;
            bool act = false;
            if (j < end) {
              const int32_t v = g.colidx[j];
              act = bit_test(Ap, v);
              if (CHURN && act)
                act = !churn_dropped((uint32_t)(p.round - 1), gidx(g, u), gidx(g, v),
                                     p.churn_thr, p.cseed_lo, p.cseed_hi);
              srow = GOSSIP ? (uint32_t)j : (uint32_t)v;
            }
            uint64_t m = __ballot(act);
            while (m) {
              uint32_t sv[8];
              bool ok[8];
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                ok[k] = m != 0ull;
                if (m) {
                  const int idx = __builtin_ctzll(m);
                  m &= m - 1ull;
                  sv[k] = (uint32_t)__builtin_amdgcn_readlane((int)srow, idx);
                } else {
                  sv[k] = 0u;
                }
              }
              uint64_t x[8];
#pragma unroll
              for (int k = 0; k < 8; ++k)
                x[k] = (ok[k] && need) ? Src[(int64_t)sv[k] * W + w] : 0ull;
#pragma unroll
              for (int k = 0; k < 8; ++k) acc |= x[k];
            }
          }
        }
        const uint64_t nw = acc & need;
        const bool any = __ballot(nw != 0ull) != 0ull;
        row_new |= any;
        if (__ballot(valid && (s | nw) != fm)) row_full = false;
        if (nw) st_prow(&st.seen[u * W + w], s | nw);
        // single-slice rows are written only when active; multi-slice rows always (a row
        // must be whole whenever its A bit is set)
        if (valid && (any || nslices > 1)) st_prow(&Fc[u * W + w], nw);
        if (nw) {
          const uint64_t pc = (uint64_t)__popcll(nw);
          c[ST_NEW] += pc;
          c[ST_RELAYS] += pc * per_bit;
          c[ST_ACTIVE_W] += 1;
          c[ST_WEDGES] += deg;
        }
      }
      if (row_new) {
        aw |= 1u << b;
        if (lane == 0) {
          c[ST_ACTIVE_V] += 1;
          c[ST_DEG_ACT] += deg;
        }
      }
      if (row_full) sat |= 1u << b;
    }
    if (lane == 0) {
      put_active(st.A[cur], task, aw, p);
      if (sat != sat0) st.S[task] = sat;
    }
  }
  flush_stats(st.stats, c, lane);
}


// One target's prefetch stage for k_pull1: row range, seen word, first 64 neighbour slots.
struct PullStage {
  int b;            // target index in the task (-1 = none)
  int64_t beg, end; // slot range
  uint64_t s;       // this lane's seen word
  int32_t v;        // this lane's neighbour (first chunk)
  uint32_t r;       // its source row (flood: v, gossip: the slot itself)
  bool act;         // neighbour active (and its send not lost); set by resolve() at use
  uint32_t aword;   // the neighbour's word of the activity bitmap, as loaded
  uint64_t mr;      // fused: active slots (of the first 64) not yet gathered
  uint64_t am;      // packed E rows: the neighbour's active-word mask
  uint32_t rv;      // fused gossip: receiver slot rev[j] of this lane's connection
};

// One target's prefetch stage for k_gossip_fused: as PullStage, with 32-bit peer and slot ids
// (gossip slot ids are uint32: rev[]) -- the fused kernel's scalar registers are the scarce ones.
// Is word w of v's frontier row live?  Packed rows (AW planes, W <= 64): iff bit w of its AW mask
// (rows written with RoundParams::store_f == 2 hold stale words elsewhere); else every word.
__device__ __forceinline__ bool aw_has(const uint64_t* __restrict__ AW, int64_t v, int w) {
  return !AW || ((ldc(AW + v) >> w) & 1ull);
}

struct FusedStage {
  int32_t u;        // the target peer (-1: none)
  uint32_t beg, end;
  uint64_t s;
  int32_t v;        // (the E row of slot j is row j itself: no per-lane row id is kept)
  uint32_t aword;
  uint64_t mr;
  uint64_t am;
  uint32_t rv;
};

// Word `lane` of a source row.  Packed E rows (gossip, st.AW) hold only the sender's active
// words in order: word w sits at position popcount(am & ((1 << w) - 1)), absent if bit w of am
// is clear (the sender had nothing in that word: the mask is zero).
__device__ __forceinline__ uint64_t src_word(const uint64_t* __restrict__ Src, uint32_t row,
                                             int W, int lane, bool packed, uint64_t am,
                                             bool want) {
  if (!packed) return want ? at_row(Src, row, W)[lane] : 0ull;
  const bool here = want && ((am >> lane) & 1ull);
  const int pos = __popcll(am & ((1ull << lane) - 1ull));
  return here ? at_row(Src, row, W)[pos] : 0ull;
}


// Packed src_word with the lane set given as a wave-uniform mask: h = the sender's active
// words (am) & the lanes that still need a word, so the exec mask comes straight from SGPRs
// (inverse ballot) and the packed position is two mbcnt -- no per-lane bit tests.
__device__ __forceinline__ uint64_t src_word_m(const uint64_t* __restrict__ Src, uint32_t row,
                                               int W, uint64_t am, uint64_t h) {
  uint64_t x = 0ull;
  if (__builtin_amdgcn_inverse_ballot_w64(h)) {
    const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
    // (row is wave-uniform: a 32 x 32 -> 64 scalar product, at_row, instead of an int64 one)
#if P2PG_NT_LOADS
    x = __builtin_nontemporal_load(at_row(Src, row, W) + pos);
#else
    x = at_row(Src, row, W)[pos];
#endif
  }
  return x;
}

// Two packed E-row slices per load for rows of W <= 32 words (k_gossip_fused<.., HALF>): lanes
// 0-31 read slot row r0, lanes 32-63 slot row r1, each at its word's packed position (m0 / m1 =
// the two senders' active words, h0 / h1 = the words to read).  A one-slot load leaves half the
// wave idle at these widths, and every slot costs the same wave-level setup.
__device__ __forceinline__ uint64_t src_word_pair(const uint64_t* __restrict__ Src, uint32_t r0,
                                                  uint32_t r1, int W, uint32_t m0, uint32_t m1,
                                                  uint32_t h0, uint32_t h1) {
  uint64_t x = 0ull;
  if (__builtin_amdgcn_inverse_ballot_w64((uint64_t)h0 | ((uint64_t)h1 << 32))) {
    const bool lo = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) < 32u;
    const uint32_t pos = __builtin_amdgcn_mbcnt_hi(m1, __builtin_amdgcn_mbcnt_lo(lo ? m0 : 0u, 0u));
    const uint32_t row = lo ? r0 : r1;  // (per lane: a 32 x 32 -> 64 address, at_row)
#if P2PG_NT_LOADS
    x = __builtin_nontemporal_load(at_row(Src, row, W) + pos);
#else
    x = at_row(Src, row, W)[pos];
#endif
  }
  return x;
}

// Same computation as k_pull for W <= 64 (one row slice), software-pipelined two targets
// deep so that a target costs ~one memory round trip instead of five: the task's 33 row
// offsets come in one load; target t+2's seen word and first neighbour chunk are issued, and
// target t+1's activity gather (A bits of its neighbours) is issued, before target t's rows
// are loaded, and all three wait together.  Hub targets (g.H) are left to k_pull_hub_*.
template <bool CHURN, bool GOSSIP>
#ifndef P2PG_PULL_WAVES
#define P2PG_PULL_WAVES 1
#endif
__global__ __launch_bounds__(256, P2PG_PULL_WAVES) void k_pull1(DevGraph g, DevState st,
                                                                RoundParams p) {
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int64_t V = g.V;
  const int W = st.W;
  const int cur = p.round & 1, prv = cur ^ 1;
  const uint64_t* __restrict__ Src = GOSSIP ? st.E[prv] : st.F[prv];
  uint64_t* __restrict__ Fc = st.F[cur];
  const uint32_t* __restrict__ Ap = st.A[prv];
  const uint64_t* __restrict__ AWp = GOSSIP ? st.AW[prv] : nullptr;
  const bool packed = GOSSIP && AWp != nullptr;
  const int64_t ntasks = (V + 31) >> 5;
  const bool valid = lane < W;
  const uint64_t fm = valid ? full_mask(lane, W, st.M) : 0ull;
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};

  for (int64_t task = (int64_t)blockIdx.x * WPB + wib; task < ntasks;
       task += (int64_t)gridDim.x * WPB) {
    const int64_t u0 = task << 5;
    const uint32_t sat0 = st.S[task];
    uint32_t todo = ~sat0 & phase_mask(p, task);
    if (g.H) todo &= ~g.H[task];  // hubs: k_pull_hub_* items
    if (V - u0 < 32) todo &= (1u << (V - u0)) - 1u;
    if (!todo) {
      if (lane == 0 && p.phase != 1) st.A[cur][task] = 0u;
      continue;
    }
    int64_t rp = 0;
    if (lane <= 32 && u0 + lane <= V) rp = g.rowptr[u0 + lane];

    auto issue = [&](PullStage& q, int b) {
      q.b = b;
      q.act = false;
      q.v = 0;
      q.r = 0;
      q.s = 0;
      if (b < 0) return;
      q.beg = readlane64(rp, b);
      q.end = readlane64(rp, b + 1);
      if (valid) q.s = st.seen[(u0 + b) * W + lane];
      const int64_t j = q.beg + lane;
      if (j < q.end) {
        q.v = g.colidx[j];
        q.r = GOSSIP ? (uint32_t)j : (uint32_t)q.v;
      }
    };
    // loads only: the bit is tested by resolve() where it is used, so the wave does not wait
    // for these loads here (their vmcnt wait would also cover every younger load in flight)
    auto activity = [&](PullStage& q) {
      if (q.b < 0) return;
      const int64_t j = q.beg + lane;
      q.am = 0;
      q.aword = 0;
      if (j < q.end) {
        // issued with (not after) the activity word: both depend only on the neighbour id
        if (packed) q.am = AWp[q.v];
        q.aword = Ap[q.v >> 5];
      }
    };
    auto resolve = [&](PullStage& q) {
      const int64_t j = q.beg + lane;
      bool a = j < q.end && ((q.aword >> (q.v & 31)) & 1u);
      if (CHURN && a)
        a = !churn_dropped((uint32_t)(p.round - 1), gidx(g, u0 + q.b), gidx(g, q.v), p.churn_thr,
                           p.cseed_lo, p.cseed_hi);
      q.act = a;
    };
    auto next_bit = [](uint32_t& t) -> int {
      if (!t) return -1;
      const int b = __builtin_ctz(t);
      t &= t - 1u;
      return b;
    };

    uint32_t rest = todo;
    PullStage s1, s2, s3;
    issue(s1, next_bit(rest));
    issue(s2, next_bit(rest));
    activity(s1);
    uint32_t aw = 0, sat = sat0;
    while (s1.b >= 0) {
      issue(s3, next_bit(rest));
      activity(s2);
      const int64_t u = u0 + s1.b;
      const uint64_t deg = (uint64_t)(s1.end - s1.beg);
      const uint64_t need = fm & ~s1.s;
      uint64_t acc = 0;
      if (__ballot(need != 0ull)) {
        resolve(s1);
        uint64_t m = __ballot(s1.act);
        uint32_t srow = s1.r;
        uint64_t sam = s1.am;
        int64_t cb = s1.beg;
        for (;;) {
          while (m) {
            uint32_t sv[8];
            uint64_t am[8];
            bool ok[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              ok[k] = m != 0ull;
              am[k] = 0ull;
              if (m) {
                const int idx = __builtin_ctzll(m);
                m &= ~(1ull << idx);
                sv[k] = (uint32_t)__builtin_amdgcn_readlane((int)srow, idx);
                if (packed) am[k] = (uint64_t)readlane64((int64_t)sam, idx);
              } else {
                sv[k] = 0u;
              }
            }
            uint64_t x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
              x[k] = src_word(Src, sv[k], W, lane, packed, am[k], ok[k] && need);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc |= x[k];
          }
          cb += 64;
          if (cb >= s1.end) break;
          const int64_t j = cb + lane;  // further chunks of a wide row: serial
          bool a = false;
          srow = 0;
          sam = 0;
          if (j < s1.end) {
            const int32_t v = g.colidx[j];
            srow = GOSSIP ? (uint32_t)j : (uint32_t)v;
            a = bit_test(Ap, v);
            if (CHURN && a)
              a = !churn_dropped((uint32_t)(p.round - 1), gidx(g, u), gidx(g, v), p.churn_thr,
                                 p.cseed_lo, p.cseed_hi);
            if (packed && a) sam = AWp[v];
          }
          m = __ballot(a);
        }
      }
      const uint64_t nw = acc & need;
      const bool any = __ballot(nw != 0ull) != 0ull;
      if (nw) {
        st_prow(at_row(st.seen, u, W) + lane, s1.s | nw);
        const uint64_t pc = (uint64_t)__popcll(nw);
        const uint64_t per_bit = GOSSIP ? (deg < (uint64_t)p.fanout ? deg : (uint64_t)p.fanout)
                                        : deg - 1;
        c[ST_NEW] += pc;
        c[ST_RELAYS] += pc * per_bit;
        c[ST_ACTIVE_W] += 1;
        c[ST_WEDGES] += deg;
      }
      if (any) {
        if (valid) st_prow(at_row(Fc, u, W) + lane, nw);
        aw |= 1u << s1.b;
        const uint64_t wm = __ballot(nw != 0ull);
        if (lane == 0) {
          if (GOSSIP && st.AW[cur]) st.AW[cur][u] = wm;
          c[ST_ACTIVE_V] += 1;
          c[ST_DEG_ACT] += deg;
        }
      }
      if (!__ballot(valid && (s1.s | nw) != fm)) sat |= 1u << s1.b;
      s1 = s2;
      s2 = s3;
    }
    if (lane == 0) {
      put_active(st.A[cur], task, aw, p);
      if (sat != sat0) st.S[task] = sat;
    }
  }
  flush_stats(st.stats, c, lane);
}

// Hub targets of the pull (deg > HUB_T), part 1: one wave per (hub, HUB_CHUNK-slot chunk)
// ORs that chunk's active source rows into a partial row.
template <bool CHURN, bool GOSSIP>
__global__ __launch_bounds__(256) void k_pull_hub_partial(DevGraph g, DevState st,
                                                          RoundParams p, HubPlan hp) {
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int W = st.W;
  const int prv = (p.round & 1) ^ 1;
  const uint64_t* __restrict__ Src = GOSSIP ? st.E[prv] : st.F[prv];
  const uint32_t* __restrict__ Ap = st.A[prv];
  const uint64_t* __restrict__ AWp = GOSSIP ? st.AW[prv] : nullptr;
  const bool packed = GOSSIP && AWp != nullptr;
  const bool valid = lane < W;
  const uint64_t fm = valid ? full_mask(lane, W, st.M) : 0ull;
  for (int64_t it = (int64_t)blockIdx.x * WPB + wib; it < hp.n_items;
       it += (int64_t)gridDim.x * WPB) {
    const int64_t item = hp.items[it];
    const int64_t u = item >> 32;
    const int64_t chunk = item & 0xFFFFFFFFll;
    const int64_t rb = g.rowptr[u], re = g.rowptr[u + 1];
    const int64_t beg = rb + chunk * HUB_CHUNK;
    const int64_t end = beg + HUB_CHUNK < re ? beg + HUB_CHUNK : re;
    const uint64_t need = valid ? fm & ~at_row(st.seen, u, W)[lane] : 0ull;
    uint64_t acc = 0;
    if (__ballot(need != 0ull) && !bit_test(st.S, u)) {
      for (int64_t cb = beg; cb < end; cb += 64) {
        const int64_t j = cb + lane;
        uint32_t srow = 0;
        uint64_t sam = 0;
        bool a = false;
        if (j < end) {
          const int32_t v = g.colidx[j];
          srow = GOSSIP ? (uint32_t)j : (uint32_t)v;
          a = bit_test(Ap, v);
          if (CHURN && a)
            a = !churn_dropped((uint32_t)(p.round - 1), gidx(g, u), gidx(g, v), p.churn_thr,
                               p.cseed_lo, p.cseed_hi);
          if (packed && a) sam = AWp[v];
        }
        uint64_t m = __ballot(a);
        while (m) {
          uint32_t sv[8];
          uint64_t am[8];
          bool ok[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            ok[k] = m != 0ull;
            am[k] = 0ull;
            if (m) {
              const int idx = __builtin_ctzll(m);
              m &= m - 1ull;
              sv[k] = (uint32_t)__builtin_amdgcn_readlane((int)srow, idx);
              if (packed) am[k] = (uint64_t)readlane64((int64_t)sam, idx);
            } else {
              sv[k] = 0u;
            }
          }
          uint64_t x[8];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            x[k] = src_word(Src, sv[k], W, lane, packed, am[k], ok[k] && need);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc |= x[k];
        }
      }
    }
    hp.partial[it * 64 + lane] = acc;
  }
}

// Hub targets, part 2: one wave per hub ORs its partial rows, dedups against seen and writes
// the frontier row; A / S bits by atomicOr (the main pull kernel stored those words whole).
// The same partial rows with the hub's adjacency segment staged in LDS (north_star: "LDS-staged
// high-degree adjacency segments"): one 256-thread block per (hub, HUB_CHUNK-slot) item.  All 256
// threads load the chunk's neighbour ids, activity (and churn) and packed-word masks at once -- one
// memory trip for the whole segment instead of one per 64-slot window of a single wave -- and
// compact the active slots into an LDS list (any order: the rows are ORed); then the 4 waves
// gather the listed rows (lane = word, 8 in flight) and their ORs are folded through LDS.
// The default since round 4 (A/B against k_pull_hub_partial).
template <bool CHURN, bool GOSSIP>
__global__ __launch_bounds__(256) void k_pull_hub_lds(DevGraph g, DevState st, RoundParams p,
                                                      HubPlan hp) {
  static_assert(HUB_CHUNK % 256 == 0, "whole slots per thread");
  __shared__ uint32_t s_row[HUB_CHUNK];   // source row: slot j (gossip, receiver-major E) or v
  __shared__ uint64_t s_am[HUB_CHUNK];    // its packed-word mask (gossip, packed E)
  __shared__ uint64_t s_acc[WPB][64];
  __shared__ uint32_t s_n;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wib = wave_in_block();
  const int W = st.W;
  const int prv = (p.round & 1) ^ 1;
  const uint64_t* __restrict__ Src = GOSSIP ? st.E[prv] : st.F[prv];
  const uint32_t* __restrict__ Ap = st.A[prv];
  const uint64_t* __restrict__ AWp = GOSSIP ? st.AW[prv] : nullptr;
  const bool packed = GOSSIP && AWp != nullptr;
  const bool valid = lane < W;
  const uint64_t fm = valid ? full_mask(lane, W, st.M) : 0ull;
  for (int64_t it = blockIdx.x; it < hp.n_items; it += gridDim.x) {
    const int64_t item = hp.items[it];
    const int64_t u = item >> 32;
    const int64_t chunk = item & 0xFFFFFFFFll;
    const int64_t rb = g.rowptr[u], re = g.rowptr[u + 1];
    const int64_t beg = rb + chunk * HUB_CHUNK;
    const int64_t end = beg + HUB_CHUNK < re ? beg + HUB_CHUNK : re;
    const uint64_t need = valid ? fm & ~at_row(st.seen, u, W)[lane] : 0ull;
    // the same for every wave of the block (same hub): skip a saturated or full hub row
    const bool run = __ballot(need != 0ull) && !bit_test(st.S, u);
    if (tid == 0) s_n = 0u;
    __syncthreads();
    if (run) {
#pragma unroll
      for (int k0 = 0; k0 < HUB_CHUNK; k0 += 256) {
        const int64_t j = beg + k0 + tid;
        if (j < end) {
          const int32_t v = g.colidx[j];
          bool a = bit_test(Ap, v);
          if (CHURN && a)
            a = !churn_dropped((uint32_t)(p.round - 1), gidx(g, u), gidx(g, v), p.churn_thr,
                               p.cseed_lo, p.cseed_hi);
          if (a) {
            const uint32_t at = atomicAdd(&s_n, 1u);
            s_row[at] = GOSSIP ? (uint32_t)j : (uint32_t)v;
            s_am[at] = packed ? AWp[v] : 0ull;
          }
        }
      }
    }
    __syncthreads();
    const uint32_t n = s_n;
    uint64_t acc = 0;
    for (uint32_t i0 = (uint32_t)wib * 8u; i0 < n; i0 += WPB * 8u) {
      uint64_t x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t i = i0 + (uint32_t)k;
        const bool ok = i < n;
        x[k] = src_word(Src, ok ? s_row[i] : 0u, W, lane, packed, ok ? s_am[i] : 0ull, ok && need);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc |= x[k];
    }
    s_acc[wib][lane] = acc;
    __syncthreads();
    if (wib == 0) {
      uint64_t r = 0;
#pragma unroll
      for (int w = 0; w < WPB; ++w) r |= s_acc[w][lane];
      hp.partial[it * 64 + lane] = r;
    }
    __syncthreads();  // s_n / s_row / s_acc are rewritten by the next item
  }
}

// part 1 of the hub pull: the LDS-staged kernel (c4 interleaved A/B, profiles/r04/ab_hub_lds.txt:
// fused rounds 211.8 -> 210.9 ms per step); P2PG_HUB_LDS=0 keeps one wave per item
template <bool CHURN, bool GOSSIP>
void launch_hub_partial(const DevGraph& g, const DevState& st, const RoundParams& p,
                        const HubPlan& hp, hipStream_t s) {
  static const bool lds = [] {
    const char* e = std::getenv("P2PG_HUB_LDS");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  if (lds)
    hipLaunchKernelGGL((k_pull_hub_lds<CHURN, GOSSIP>),
                       dim3((unsigned)std::min<int64_t>(hp.n_items, 65535)), dim3(256), 0, s, g, st,
                       p, hp);
  else
    hipLaunchKernelGGL((k_pull_hub_partial<CHURN, GOSSIP>), dim3(grid_tasks(hp.n_items)),
                       dim3(256), 0, s, g, st, p, hp);
}

template <bool GOSSIP>
__global__ __launch_bounds__(256) void k_pull_hub_finalize(DevGraph g, DevState st,
                                                           RoundParams p, HubPlan hp) {
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int W = st.W;
  const int cur = p.round & 1;
  const bool valid = lane < W;
  const uint64_t fm = valid ? full_mask(lane, W, st.M) : 0ull;
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t h = (int64_t)blockIdx.x * WPB + wib; h < hp.n_hubs;
       h += (int64_t)gridDim.x * WPB) {
    const int64_t u = hp.hubs[h];
    if (bit_test(st.S, u)) continue;
    uint64_t acc = 0;
    for (int64_t it = hp.item_begin[h]; it < hp.item_begin[h + 1]; ++it)
      acc |= hp.partial[it * 64 + lane];
    const uint64_t s = valid ? at_row(st.seen, u, W)[lane] : 0ull;
    const uint64_t nw = acc & fm & ~s;
    const uint64_t deg = (uint64_t)(g.rowptr[u + 1] - g.rowptr[u]);
    if (nw) {
      st_prow(at_row(st.seen, u, W) + lane, s | nw);
      const uint64_t pc = (uint64_t)__popcll(nw);
      const uint64_t per_bit = GOSSIP ? (deg < (uint64_t)p.fanout ? deg : (uint64_t)p.fanout)
                                      : deg - 1;
      c[ST_NEW] += pc;
      c[ST_RELAYS] += pc * per_bit;
      c[ST_ACTIVE_W] += 1;
      c[ST_WEDGES] += deg;
    }
    if (__ballot(nw != 0ull)) {
      if (valid) st_prow(&st.F[cur][u * W + lane], nw);
      const uint64_t wm = __ballot(nw != 0ull);
      if (lane == 0) {
        if (GOSSIP && st.AW[cur]) st.AW[cur][u] = wm;
        atomicOr(&st.A[cur][u >> 5], 1u << (u & 31));
        c[ST_ACTIVE_V] += 1;
        c[ST_DEG_ACT] += deg;
      }
    }
    if (!__ballot(valid && (s | nw) != fm) && lane == 0) atomicOr(&st.S[u >> 5], 1u << (u & 31));
  }
  flush_stats(st.stats, c, lane);
}

// ---------------------------------------------------------------------------------------
// Gossip, round r >= 1 after a sparse round: consume the row-atomic pushes of round r-1
// (next[r&1], touched bitmap T[r&1]), dedup against seen, write the round-r frontier row and
// A bit, clear what was consumed.  Relays: min(k, deg) per first receipt.
__global__ __launch_bounds__(256) void k_gossip_update(DevGraph g, DevState st,
                                                        RoundParams p) {
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int64_t V = g.V;
  const int W = st.W;
  const int cur = p.round & 1;
  uint64_t* __restrict__ nx = st.next[cur];
  uint64_t* __restrict__ Fc = st.F[cur];
  const int64_t ntasks = (V + 31) >> 5;
  const int nslices = (W + 63) >> 6;
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};

  for (int64_t task = (int64_t)blockIdx.x * WPB + wib; task < ntasks;
       task += (int64_t)gridDim.x * WPB) {
    const uint32_t tw0 = st.T[cur][task];
    uint32_t tw = tw0 & phase_mask(p, task);
    uint32_t aw = 0;
    if (tw && lane == 0) st.T[cur][task] = tw0 & ~tw;  // consumed (the other phase's bits stay)
    while (tw) {
      const int b = __builtin_ctz(tw);
      tw &= tw - 1u;
      const int64_t u = (task << 5) + b;
      const int64_t deg = g.rowptr[u + 1] - g.rowptr[u];
      // relays per first receipt: gossip min(k, deg); flood (rows materialized by a topology
      // update) deg - 1, the sender's connection being excluded (node.py:106-112)
      const uint64_t fan = p.mode == 0 ? (uint64_t)(deg > 0 ? deg - 1 : 0)
                                       : (uint64_t)(deg < p.fanout ? deg : p.fanout);
      bool row_new = false;
      for (int sl = 0; sl < nslices; ++sl) {
        const int w = sl * 64 + lane;
        const bool valid = w < W;
        uint64_t x = 0, s = 0;
        if (valid) {
          x = nx[u * W + w];
          if (x) {
            st_prow(&nx[u * W + w], 0ull);
            s = st.seen[u * W + w];
            c[ST_AUX] += 1;  // touched (pushed-to) words consumed
          }
        }
        const uint64_t nw = x & ~s;
        const uint64_t wm = __ballot(nw != 0ull);
        const bool any = wm != 0ull;
        row_new |= any;
        if (any && nslices == 1 && st.AW[cur] && lane == 0) st.AW[cur][u] = wm;
        if (nw) st_prow(&st.seen[u * W + w], s | nw);
        if (valid && (any || nslices > 1)) st_prow(&Fc[u * W + w], nw);
        if (nw) {
          const uint64_t pc = (uint64_t)__popcll(nw);
          c[ST_NEW] += pc;
          c[ST_RELAYS] += pc * fan;
          c[ST_ACTIVE_W] += 1;
          c[ST_WEDGES] += (uint64_t)deg;
        }
      }
      if (row_new) {
        aw |= 1u << b;
        if (lane == 0) {
          c[ST_ACTIVE_V] += 1;
          c[ST_DEG_ACT] += (uint64_t)deg;
        }
      }
    }
    if (lane == 0) put_active(st.A[cur], task, aw, p);
  }
  flush_stats(st.stats, c, lane);
}

// The same update for single-slice rows (W <= 64), software-pipelined over the touched peers
// of a wave's tasks: the push row of peer t+2 and the seen words of t+1 (where t+1's push row
// is nonzero) are in flight while t is consumed, so a touched peer costs one memory round trip
// instead of two in sequence; the next task's touched word is a scalar load issued one task
// ahead (only this wave writes a task's T word, after reading it).  Same results as
// k_gossip_update (every gossip test runs it).
struct UpdStage {
  int64_t u;   // touched peer (-1: none)
  int64_t u2;  // PAIR / DUAL: a second touched peer of the same task (-1: none)
  uint64_t x;  // this lane's push word
  uint64_t s;  // this lane's seen word (where x != 0)
  uint64_t x2; // DUAL: the second peer's push word and seen word
  uint64_t s2;
};

// NP = 1: one touched peer per stage, lane = word.
// NP = 2, PAIR (W <= 32): two touched peers of a task per stage, lanes 0-31 the first, 32-63 the
//   second (one peer per wave leaves half the wave idle at these widths and pays the per-peer wave
//   work once per peer).
// NP = 3, DUAL (W <= 64): two touched peers of a task per stage, lane = word of both (two words
//   per lane).  The update is latency-bound: every stage waits for one memory round trip (its
//   rows' loads) and a wave consumed ONE peer per trip (c4 round 9: ~1.3 us per peer per wave at
//   ~3.5 TB/s); two rows per trip halve the trips.
template <int NP = 1>
__global__ __launch_bounds__(256) void k_gossip_update1(DevGraph g, DevState st, RoundParams p) {
  constexpr bool PAIR = NP == 2, DUAL = NP == 3;
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int64_t V = g.V;
  const int W = st.W;
  const int cur = p.round & 1;
  uint64_t* __restrict__ nx = st.next[cur];
  uint64_t* __restrict__ Fc = st.F[cur];
  uint32_t* __restrict__ Tc = st.T[cur];
  const int64_t ntasks = (V + 31) >> 5;
  const int hl = PAIR ? lane >> 5 : 0;      // PAIR: which peer of the stage this lane serves
  const int wl = PAIR ? lane & 31 : lane;   // ... and its word
  const bool valid = wl < W;
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};

  // This wave's tasks are w0 + i * tstride (i = 0, 1, ..), taken 64 at a time into a table (lane
  // l: task i = tb + l), one vector load per 64 tasks: a one-task-at-a-time scan paid a
  // dependent load per task (~76 per wave on config 4), i.e. ~40 us for a round with a few
  // hundred touched peers; now two.  The table's empty tasks get their activity word cleared and
  // its touched ones their T word consumed (only this wave reads them) when it is loaded.
  const int64_t tstride = (int64_t)gridDim.x * WPB;
  const int64_t w0 = (int64_t)blockIdx.x * WPB + wib;
  int64_t tb = 0;        // table index i of lane 0 of the next table
  uint64_t tmask = 0;    // table lanes whose touched task is not issued yet
  uint32_t tval = 0;     // lane l: its task's touched peers (phase-filtered)
  int64_t it_task = 0;
  uint32_t it_rest = 0;
  auto load_table = [&]() -> bool {
    for (;;) {
      if (w0 + tb * tstride >= ntasks) return false;
      const int64_t t = w0 + (tb + lane) * tstride;
      const bool ok = t < ntasks;
      const uint32_t tw0 = ok ? Tc[t] : 0u;
      const uint32_t tw = ok ? tw0 & phase_mask(p, t) : 0u;
      if (ok && !tw && p.phase != 1) st.A[cur][t] = 0u;  // put_active(.., 0, ..)
      if (tw) Tc[t] = tw0 & ~tw;  // consumed (the other phase's bits stay)
      tval = tw;
      tmask = __ballot(tw != 0u);
      tb += 64;
      if (tmask) return true;
    }
  };
  auto next_peer = [&]() -> int64_t {
    while (!it_rest) {
      if (!tmask && !load_table()) return -1;
      const int l = __builtin_ctzll(tmask);
      tmask &= tmask - 1ull;
      it_task = w0 + (tb - 64 + l) * tstride;
      it_rest = (uint32_t)__builtin_amdgcn_readlane((int)tval, l);
    }
    const int b = __builtin_ctz(it_rest);
    it_rest &= it_rest - 1u;
    return (it_task << 5) + b;
  };
  auto issue_x = [&](UpdStage& q) {
    q.u = next_peer();
    q.u2 = ((PAIR || DUAL) && q.u >= 0 && it_rest) ? next_peer() : -1;  // never across a task boundary
    q.x = 0;
    q.s = 0;
    q.x2 = 0;
    q.s2 = 0;
    const int64_t me = hl ? q.u2 : q.u;
    if (me >= 0 && valid) q.x = at_row(nx, me, W)[wl];
    if (DUAL && q.u2 >= 0 && valid) q.x2 = at_row(nx, q.u2, W)[wl];
  };
  auto issue_s = [&](UpdStage& q) {
    const int64_t me = hl ? q.u2 : q.u;
    if (me >= 0 && q.x) q.s = at_row(st.seen, me, W)[wl];
    if (DUAL && q.u2 >= 0 && q.x2) q.s2 = at_row(st.seen, q.u2, W)[wl];
  };

  int64_t ct = -1;  // task of the consumed peers
  uint32_t aw = 0;
  auto finish_task = [&]() {
    if (ct >= 0 && lane == 0) put_active(st.A[cur], ct, aw, p);
    aw = 0;
  };
  // one peer u (lanes: its words x / seen s) of this lane's stage
  // (wm_all: the stage's ballot of new words; PAIR: this lane's half of it is its peer's)
  auto consume_one = [&](int64_t u, int64_t deg, uint64_t x, uint64_t s, uint64_t wm_all, int shift) {
    // relays per first receipt: gossip min(k, deg); flood (rows materialized by a topology
    // update) deg - 1, the sender's connection being excluded (node.py:106-112)
    const uint64_t fan = p.mode == 0 ? (uint64_t)(deg > 0 ? deg - 1 : 0)
                                     : (uint64_t)(deg < p.fanout ? deg : p.fanout);
    if (x) {
      st_prow(at_row(nx, u, W) + wl, 0ull);
      c[ST_AUX] += 1;  // touched (pushed-to) words consumed
    }
    const uint64_t nw = x & ~s;
    const uint64_t wm = PAIR ? (wm_all >> shift) & 0xFFFFFFFFull : wm_all;
    if (wm && st.AW[cur] && wl == 0) st.AW[cur][u] = wm;
    if (nw) st_prow(at_row(st.seen, u, W) + wl, s | nw);
    if (valid && wm && (p.store_f != 2 || nw)) st_prow(at_row(Fc, u, W) + wl, nw);  // (2: AW-valid rows)
    if (nw) {
      const uint64_t pc = (uint64_t)__popcll(nw);
      c[ST_NEW] += pc;
      c[ST_RELAYS] += pc * fan;
      c[ST_ACTIVE_W] += 1;
      c[ST_WEDGES] += (uint64_t)deg;
    }
    if (wm && wl == 0) {
      c[ST_ACTIVE_V] += 1;
      c[ST_DEG_ACT] += (uint64_t)deg;
    }
  };
  auto consume = [&](const UpdStage& q) {
    if ((q.u >> 5) != ct) {
      finish_task();
      ct = q.u >> 5;
    }
    const int64_t deg1 = ldc(g.rowptr + q.u + 1) - ldc(g.rowptr + q.u);
    const int64_t deg2 = (PAIR || DUAL) && q.u2 >= 0 ? ldc(g.rowptr + q.u2 + 1) - ldc(g.rowptr + q.u2) : 0;
    const uint64_t nw1 = q.x & ~q.s;
    const uint64_t wmb = __ballot(nw1 != 0ull);
    if (PAIR) {
      // lanes 0-31 serve q.u, lanes 32-63 q.u2
      const uint64_t wm1 = wmb & 0xFFFFFFFFull, wm2 = wmb >> 32;
      consume_one(hl ? q.u2 : q.u, hl ? deg2 : deg1, q.x, q.s, wmb, hl ? 32 : 0);
      if (wm1) aw |= 1u << (q.u & 31);
      if (wm2) aw |= 1u << (q.u2 & 31);
      return;
    }
    consume_one(q.u, deg1, q.x, q.s, wmb, 0);
    if (wmb) aw |= 1u << (q.u & 31);
    if (DUAL && q.u2 >= 0) {
      const uint64_t wmb2 = __ballot((q.x2 & ~q.s2) != 0ull);
      consume_one(q.u2, deg2, q.x2, q.s2, wmb2, 0);
      if (wmb2) aw |= 1u << (q.u2 & 31);
    }
  };
  // three stages rotate by unrolling (a register copy of a load in flight would wait for it)
  auto step = [&](UpdStage& a, UpdStage& b, UpdStage& cc) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): a's seen words and b's push row landed
    issue_s(b);
    issue_x(cc);
    consume(a);
  };
  UpdStage sA, sB, sC;
  issue_x(sA);
  issue_x(sB);
  issue_s(sA);
  for (;;) {
    if (sA.u < 0) break;
    step(sA, sB, sC);
    if (sB.u < 0) break;
    step(sB, sC, sA);
    if (sC.u < 0) break;
    step(sC, sA, sB);
  }
  finish_task();
  flush_stats(st.stats, c, lane);
}

// The same update for narrow rows (W <= 32: one rank's share of a message split): G = 64 / WP
// touched peers per wave pass, lane = (peer g, word w), WP = W rounded up to a power of two, so
// the per-peer fixed work (ballots, counters, stores) is shared by G peers.  The touched peers
// of a task word are picked by select-nth-bit; the next task's word is a scalar load issued one
// task ahead.  Same results as k_gossip_update.
template <int LW>
__global__ __launch_bounds__(256) void k_gossip_update_g(DevGraph g, DevState st, RoundParams p) {
  constexpr int WP = 1 << LW, G = 64 >> LW;
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int W = st.W;
  const int cur = p.round & 1;
  uint64_t* __restrict__ nx = st.next[cur];
  uint64_t* __restrict__ Fc = st.F[cur];
  uint32_t* __restrict__ Tc = st.T[cur];
  uint64_t* __restrict__ AWc = st.AW[cur];
  const int64_t ntasks = (g.V + 31) >> 5;
  const int grp = lane >> LW, w = lane & (WP - 1);
  const uint64_t segm = WP >= 64 ? ~0ull : (1ull << WP) - 1ull;
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t tstride = (int64_t)gridDim.x * WPB;
  int64_t task = (int64_t)blockIdx.x * WPB + wib;
  uint32_t tw_next = task < ntasks ? ldc(&Tc[task]) : 0u;
  for (; task < ntasks; task += tstride) {
    const uint32_t tw0 = tw_next;
    tw_next = task + tstride < ntasks ? ldc(&Tc[task + tstride]) : 0u;
    const uint32_t tw = tw0 & phase_mask(p, task);
    if (!tw) {
      if (lane == 0 && p.phase != 1) st.A[cur][task] = 0u;  // put_active(.., 0, ..)
      continue;
    }
    if (lane == 0) Tc[task] = tw0 & ~tw;  // consumed (the other phase's bits stay)
    const uint32_t n = (uint32_t)__popc(tw);
    uint32_t aw = 0;
    for (uint32_t pb = 0; pb < n; pb += G) {
      const uint32_t idx = pb + (uint32_t)grp;
      const bool peer = idx < n;
      const bool ok = peer && w < W;
      const int64_t u = (task << 5) + (peer ? select_bit32(tw, idx) : 0u);
      uint64_t x = 0, s = 0;
      if (ok) x = at_row(nx, u, W)[w];
      if (x) {
        s = at_row(st.seen, u, W)[w];
        st_prow(at_row(nx, u, W) + w, 0ull);
        c[ST_AUX] += 1;  // touched (pushed-to) words consumed
      }
      const uint64_t nw = x & ~s;
      const uint64_t wm = (__ballot(nw != 0ull) >> (grp * WP)) & segm;  // this peer's new words
      if (nw) st_prow(at_row(st.seen, u, W) + w, s | nw);
      if (ok && wm) st_prow(at_row(Fc, u, W) + w, nw);
      if (wm) {
        const int64_t deg = g.rowptr[u + 1] - g.rowptr[u];
        // relays per first receipt: gossip min(k, deg); flood (rows materialized by a topology
        // update) deg - 1, the sender's connection being excluded (node.py:106-112)
        const uint64_t fan = p.mode == 0 ? (uint64_t)(deg > 0 ? deg - 1 : 0)
                                         : (uint64_t)(deg < p.fanout ? deg : p.fanout);
        if (nw) {
          const uint64_t pc = (uint64_t)__popcll(nw);
          c[ST_NEW] += pc;
          c[ST_RELAYS] += pc * fan;
          c[ST_ACTIVE_W] += 1;
          c[ST_WEDGES] += (uint64_t)deg;
        }
        if (w == 0) {
          if (AWc) AWc[u] = wm;
          c[ST_ACTIVE_V] += 1;
          c[ST_DEG_ACT] += (uint64_t)deg;
        }
      }
      // distinct bits per peer: the wave sum of (w == 0 lanes' bits) is their OR
      aw |= wave_reduce_u32<false>(w == 0 && wm ? 1u << (u & 31) : 0u);
    }
    if (lane == 0) put_active(st.A[cur], task, aw, p);
  }
  flush_stats(st.stats, c, lane);
}

// The update for rows of W <= 16 words, pipelined like k_gossip_update1: G = 64 / WP touched peers
// of one task per stage (lane = (peer g, word w), WP = W rounded up to a power of two), three
// stages in flight (push rows + row offsets of t+2, seen words of t+1, consume t).  Each lane
// carries its stage peer's id, so a stage costs no scalar registers per peer.  Same results as
// k_gossip_update.
struct UpdStageG {
  int32_t t;   // task of the stage's peers (-1: no peers)
  int32_t me;  // this lane's peer (-1: none)
  uint64_t x;  // its push word
  uint64_t s;  // its seen word (where x != 0)
  uint32_t r0, r1;  // its peer's slot range (relays / wedges)
};

template <int LW>
__global__ __launch_bounds__(256) void k_gossip_update_gp(DevGraph g, DevState st, RoundParams p) {
  constexpr int WP = 1 << LW, G = 64 >> LW;
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int W = st.W;
  const int cur = p.round & 1;
  uint64_t* __restrict__ nx = st.next[cur];
  uint64_t* __restrict__ Fc = st.F[cur];
  uint32_t* __restrict__ Tc = st.T[cur];
  uint64_t* __restrict__ AWc = st.AW[cur];
  const int32_t ntasks = (int32_t)((g.V + 31) >> 5);
  const int grp = lane >> LW, w = lane & (WP - 1);
  const bool wvalid = w < W;
  const uint64_t segm = WP >= 64 ? ~0ull : (1ull << WP) - 1ull;
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};

  const int32_t tstride = (int32_t)gridDim.x * WPB;
  int32_t pf_task = (int32_t)blockIdx.x * WPB + wib;
  uint32_t pf_tw = pf_task < ntasks ? ldc(&Tc[pf_task]) : 0u;
  int32_t it_task = 0;
  uint32_t it_rest = 0;
  auto next_task = [&]() -> bool {  // make it_rest the next task's touched peers (false: none left)
    while (!it_rest) {
      const int32_t t = pf_task;
      if (t >= ntasks) return false;
      const uint32_t tw0 = pf_tw;
      pf_task = t + tstride;
      pf_tw = pf_task < ntasks ? ldc(&Tc[pf_task]) : 0u;
      const uint32_t tw = tw0 & phase_mask(p, t);
      if (!tw) {
        if (lane == 0 && p.phase != 1) st.A[cur][t] = 0u;  // put_active(.., 0, ..)
        continue;
      }
      if (lane == 0) Tc[t] = tw0 & ~tw;  // consumed (the other phase's bits stay)
      it_task = t;
      it_rest = tw;
    }
    return true;
  };
  auto issue_x = [&](UpdStageG& q) {
    q.t = -1;
    q.me = -1;
    q.x = 0;
    q.s = 0;
    q.r0 = q.r1 = 0;
    if (!next_task()) return;
    q.t = it_task;
    // up to G peers of this task, lowest first: group g takes the g-th remaining bit
    const uint32_t n = (uint32_t)__popc(it_rest);
    const uint32_t take = n < (uint32_t)G ? n : (uint32_t)G;
    if ((uint32_t)grp < take) q.me = (it_task << 5) + (int32_t)select_bit32(it_rest, (uint32_t)grp);
    // the rest of the task: its bits from the (take)-th on
    it_rest = take >= n ? 0u : it_rest & ~((1u << select_bit32(it_rest, take)) - 1u);
    if (q.me >= 0) {
      if (wvalid) q.x = at_row(nx, q.me, W)[w];
      q.r0 = (uint32_t)g.rowptr[q.me];
      q.r1 = (uint32_t)g.rowptr[q.me + 1];
    }
  };
  auto issue_s = [&](UpdStageG& q) {
    if (q.me >= 0 && q.x) q.s = at_row(st.seen, q.me, W)[w];
  };
  auto consume = [&](const UpdStageG& q) {
    const int64_t u = q.me;
    const uint64_t x = q.x, s = q.s;
    if (x) {
      st_prow(at_row(nx, u, W) + w, 0ull);
      c[ST_AUX] += 1;  // touched (pushed-to) words consumed
    }
    const uint64_t nw = x & ~s;
    const uint64_t wm = (__ballot(nw != 0ull) >> (grp * WP)) & segm;  // this peer's new words
    if (nw) st_prow(at_row(st.seen, u, W) + w, s | nw);
    if (q.me >= 0 && wvalid && wm) st_prow(at_row(Fc, u, W) + w, nw);
    uint32_t bit = 0;
    if (wm) {
      const int64_t deg = (int64_t)(q.r1 - q.r0);
      // relays per first receipt: gossip min(k, deg); flood (rows materialized by a topology
      // update) deg - 1, the sender's connection being excluded (node.py:106-112)
      const uint64_t fan = p.mode == 0 ? (uint64_t)(deg > 0 ? deg - 1 : 0)
                                       : (uint64_t)(deg < p.fanout ? deg : p.fanout);
      if (nw) {
        const uint64_t pc = (uint64_t)__popcll(nw);
        c[ST_NEW] += pc;
        c[ST_RELAYS] += pc * fan;
        c[ST_ACTIVE_W] += 1;
        c[ST_WEDGES] += (uint64_t)deg;
      }
      if (w == 0) {
        if (AWc) AWc[u] = wm;
        c[ST_ACTIVE_V] += 1;
        c[ST_DEG_ACT] += (uint64_t)deg;
        bit = 1u << (u & 31);
      }
    }
    // distinct bits per peer: the wave sum of the w == 0 lanes' bits is their OR
    return wave_reduce_u32<false>(bit);
  };
  int32_t ct = -1;  // task of the consumed stages
  uint32_t aw = 0;
  auto step = [&](UpdStageG& a, UpdStageG& b, UpdStageG& cc) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): a's seen words and b's push rows landed
    issue_s(b);
    issue_x(cc);
    if (a.t != ct) {
      if (ct >= 0 && lane == 0) put_active(st.A[cur], ct, aw, p);
      aw = 0;
      ct = a.t;
    }
    aw |= consume(a);
  };
  UpdStageG sA, sB, sC;
  issue_x(sA);
  issue_x(sB);
  issue_s(sA);
  for (;;) {
    if (sA.t < 0) break;
    step(sA, sB, sC);
    if (sB.t < 0) break;
    step(sB, sC, sA);
    if (sC.t < 0) break;
    step(sC, sA, sB);
  }
  if (ct >= 0 && lane == 0) put_active(st.A[cur], ct, aw, p);
  flush_stats(st.stats, c, lane);
}

// Messages in flight after round r = p.round - 1, as row pushes into next[p.round&1] + T bits
// (the form k_gossip_update consumes), one wave per receiver u, lane = word, serial over u's
// slots (not a hot path):
//   FLOOD = false: gossip pushes held per connection in E[r&1] (a dense round), so that the
//                  run state no longer depends on slot numbering (snapshots);
//   FLOOD = true:  flood sends of round r = the frontier rows F[r&1] of u's active neighbours
//                  (churn of round r applied), over g -- the graph they were sent on -- minus
//                  the slots a topology update removed (g.gone).
template <bool FLOOD>
__global__ __launch_bounds__(256) void k_materialize(DevGraph g, DevState st, RoundParams p) {
  const int lane = threadIdx.x & 63;
  const int W = st.W;
  const int cur = p.round & 1, prv = cur ^ 1;
  const uint64_t* __restrict__ Src = FLOOD ? st.F[prv] : st.E[prv];
  const uint32_t* __restrict__ Ap = st.A[prv];
  const uint64_t* __restrict__ AWp = FLOOD ? nullptr : st.AW[prv];
  const bool packed = AWp != nullptr;
  const int nslices = (W + 63) >> 6;
  for (int64_t u = (int64_t)blockIdx.x * WPB + wave_in_block(); u < g.V;
       u += (int64_t)gridDim.x * WPB) {
    const int64_t beg = g.rowptr[u], end = g.rowptr[u + 1];
    bool any = false;
    for (int sl = 0; sl < nslices; ++sl) {
      const int w = sl * 64 + lane;
      uint64_t acc = 0;
      for (int64_t j = beg; j < end; ++j) {
        const int32_t v = g.colidx[j];
        if (!bit_test(Ap, v)) continue;
        if (FLOOD) {
          if (g.gone && g.gone[j]) continue;
          if (p.churn_thr && churn_dropped((uint32_t)(p.round - 1), gidx(g, u), gidx(g, v),
                                           p.churn_thr, p.cseed_lo, p.cseed_hi))
            continue;
          acc |= w < W ? Src[(int64_t)v * W + w] : 0ull;
        } else {
          acc |= packed ? src_word(Src, (uint32_t)j, W, lane, true, AWp[v], true)
                        : (w < W ? Src[j * W + w] : 0ull);
        }
      }
      if (acc) st.next[cur][u * W + w] |= acc;
      any |= __ballot(acc != 0ull) != 0ull;
    }
    if (any && lane == 0) atomicOr(&st.T[cur][u >> 5], 1u << (u & 31));
  }
}


// Development builds (-DP2PG_PROF): wave clock per fused-kernel segment, summed into st.prof.
#ifdef P2PG_PROF
#define PROF_DECL uint64_t pf_[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}; uint64_t pt_ = __builtin_amdgcn_s_memtime();
#define PROF_MARK(i)                                  \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    pf_[i] += t_ - pt_;                               \
    pt_ = t_;                                         \
  } while (0)
#define PROF_FLUSH \
  if (lane == 0) for (int i_ = 0; i_ < 9; ++i_) atomicAdd(&st.prof[i_], (unsigned long long)pf_[i_]);
#define PROF_PARAMS , uint64_t* pf_, uint64_t& pt_
#define PROF_PASS , pf_, pt_
#else
#define PROF_DECL
#define PROF_MARK(i)
#define PROF_FLUSH
#define PROF_PARAMS
#define PROF_PASS
#endif

#ifndef P2PG_PICK_PAIRS
#define P2PG_PICK_PAIRS 0
#endif
#ifndef P2PG_COMPACT
#define P2PG_COMPACT 1
#endif

// LDS of one scatter wave: a GCHUNK x 64-word mask table (two 32-bit halves per word, so
// 32-bit LDS atomics) and the compacted list of active (word, bit) entries.
// Half-major rows (P2PG_TBL_HALF_MAJOR, default): connection j's row is [half][word], so the
// 64 lanes of a pick batch -- entries of ~64 different words -- OR into 64 different banks;
// with the halves adjacent ([word][half], a 64-bit LDS access per mask) words w and w+32 share
// a bank (2-way conflicts: 40-49 % of the fused kernel's LDS cycles, profiles/r01/pmc_sq_v11).
#ifndef P2PG_TBL_HALF_MAJOR
#define P2PG_TBL_HALF_MAJOR 1
#endif
struct ScatterLds {
  alignas(8) uint32_t tbl[GCHUNK * 128];
  uint16_t lst[GLIST];
};

// u32 index of half h of (connection j, word w)
__device__ __forceinline__ uint32_t tbl_ix(uint32_t j, uint32_t w, uint32_t h) {
#if P2PG_TBL_HALF_MAJOR
  return j * 128u + h * 64u + w;
#else
  return j * 128u + w * 2u + h;
#endif
}

// u32 index of list entry e = word << 6 | bit in connection 0's row
__device__ __forceinline__ uint32_t tbl_entry_ix(uint32_t e) {
  return tbl_ix(0u, e >> 6, (e >> 5) & 1u);
}

__device__ __forceinline__ uint64_t tbl_word(const ScatterLds& L, int j, int w) {
#if P2PG_TBL_HALF_MAJOR
  return ((uint64_t)L.tbl[tbl_ix(j, w, 1)] << 32) | L.tbl[tbl_ix(j, w, 0)];
#else
  return *reinterpret_cast<const uint64_t*>(&L.tbl[tbl_ix(j, w, 0)]);
#endif
}

__device__ __forceinline__ void tbl_clear(ScatterLds& L, int j, int w) {
  L.tbl[tbl_ix(j, w, 0)] = 0u;
  L.tbl[tbl_ix(j, w, 1)] = 0u;
}

// Gossip, round r >= 0: every first receipt (v, m) of round r is pushed to k Philox-chosen
// neighbours.  One wave per (source, GCHUNK-neighbour chunk):
//   1. the row slice's active bits are compacted into an LDS list (prefix sum of popcounts),
//      so the 64 lanes evaluate Philox + Floyd for equal shares of messages;
//   2. picks landing in the chunk set bits of a GCHUNK x 64-word LDS mask table (32-bit LDS
//      atomics; table = [target][word][half]: one 64-bit LDS access per (target, word) in the
//      clear and the flush);
//   3. flush, lane = word: every (target, word) mask leaves as part of one 512 B row access --
//      STORE_E = false (sparse rounds): row atomicOr into the target's next row + T bit;
//      STORE_E = true  (dense rounds):  plain store of the whole row (zeros included) into
//      E[r&1][rev(slot)], the receiver's own slot of the connection, which the next round's
//      pull then streams contiguously per receiver.
// One (source v, neighbour chunk, row slice): f = this lane's frontier word, nbr = lane j's
// neighbour nb + j is lane nbr0 + j of nbr -- its receiver slot (STORE_E) or its local id
// (row atomics).  Every
// per-source value is a scalar load or a lane of a prefetched register: a vector load here
// would make the wave wait (vmcnt) for its own in-flight row stores / atomics.
// PH: 0 = the whole push; 1 = table + picks only (the flush follows later, PH 2, with the same
// source, f and receiver slots: the fused kernel defers a short row's flush by one target).
// PART (vertex-partitioned gossip ranks, STORE_E): a receiver slot marked REV_GHOST is a ghost's
// connection -- the mask goes into the ghost's row push (next[r+1] row + T bit, exchanged after the
// round) as in a sparse round, every other one into its E slot.
template <bool CHURN, int K, bool STORE_E, int PH = 0, bool PART = false, bool DIRECT = false, class CT>
__device__ __forceinline__ void scatter_row(const DevGraph& g, const DevState& st,
                                            const RoundParams& p, ScatterLds& L, int lane,
                                            int64_t v, int64_t rb, int64_t deg, int chunk,
                                            int sl, uint64_t f, uint32_t nbr, int nbr0,
                                            CT* c PROF_PARAMS) {
  const int W = st.W;
  const int cur = p.round & 1, nxt = cur ^ 1;
  uint64_t* __restrict__ nx = st.next[nxt];
  uint32_t* __restrict__ Tn = st.T[nxt];
  uint64_t* __restrict__ Eo = st.E[cur];
  const int k = K > 0 ? K : p.fanout;
  const int nb = chunk * GCHUNK;
  const int nn = (int)(deg - nb < GCHUNK ? deg - nb : GCHUNK);
  const bool all = deg <= k;
  const int w = sl * 64 + lane;
  const bool valid = w < W;
  const uint64_t fam = __ballot(f != 0ull);  // active words of this slice
  const bool anyf = fam != 0ull;
  if (!anyf && !STORE_E) return;
  const uint32_t gv = gidx_s(g, v);
  // the source's folded Philox rounds (philox_pick: only the message varies per draw)
  const PickKey pkey = pick_key((uint32_t)p.round, gv, p.gseed_lo, p.gseed_hi);

  // Philox + Floyd for one (word, bit) entry e = word << 6 | bit of this slice, its picks ORed
  // into the LDS table (an empty mask when !ok); CHECK: picks outside this chunk are dropped.
  auto one = [&](auto check_v, uint32_t e, bool ok) {
    constexpr bool CHECK = decltype(check_v)::value;
    const uint32_t wl = e >> 6, bit = e & 63u;
    const uint32_t mg = p.msg_base + (uint32_t)((sl * 64 + (int)wl) * 64) + bit;
    uint32_t* const col = &L.tbl[tbl_entry_ix(e)];  // connection 0's (word, half)
    const uint32_t mb = ok ? 1u << (bit & 31u) : 0u;
    uint32_t pk[K > 0 ? K : 1];
    if constexpr (P2PG_PICK_FOLD && K > 0 && K <= 4)
      gossip_picks_k<K>(pkey, mg, (uint32_t)deg, pk);
    else
      gossip_picks_t<(K > 0 ? K : 1)>((uint32_t)p.round, gv, mg, (uint32_t)deg, p.gseed_lo,
                                      p.gseed_hi, pk);
#pragma unroll
    for (int q = 0; q < (K > 0 ? K : 1); ++q) {
      const uint32_t jj = pk[q] - (uint32_t)nb;
      if (!CHECK || jj < (uint32_t)nn) atomicOr(col + jj * 128u, mb);
    }
  };
  // Philox + Floyd for list entries [0, n) of this wave, picks ORed into the LDS table.
  auto pick_batch = [&](auto check_v, uint32_t n) {
    // Strided: in batch b lane l takes entry l*nbat + b.  The list is word-major (a word's
    // bits are adjacent), so the 64 entries of a batch come from ~64 different words, i.e.
    // their table atomics hit different LDS banks.  The next batch's entry is read before this
    // batch's Philox (hides the LDS trip).
    const uint32_t nbat = (n + 63) >> 6;
    const uint32_t i0 = (uint32_t)lane * nbat;
    const uint32_t cnt = i0 < n ? (n - i0 < nbat ? n - i0 : nbat) : 0u;
#if P2PG_PICK_PAIRS
    // two entries per iteration, evaluated unconditionally (the second's atomics masked when
    // past the lane's share): two independent Philox chains interleave and hide each other's
    // multiply latency
    for (uint32_t b = 0; b < cnt; b += 2) {
      const uint32_t e0 = L.lst[i0 + b];
      const bool two = b + 1 < cnt;
      const uint32_t e1 = two ? L.lst[i0 + b + 1] : e0;
      one(check_v, e0, true);
      one(check_v, e1, two);
    }
#else
    // Uniform trip count: a lane past its share evaluates a dummy entry whose table ORs carry
    // an empty mask, so the loop needs no per-lane exit bookkeeping.  i0 + b + 1 <= GLIST.
    uint32_t en = L.lst[i0];
    for (uint32_t b = 0; b < nbat; ++b) {
      const uint32_t e = en & 0x0FFFu;  // in range even when stale
      const uint32_t ni = i0 + b + 1;
      en = L.lst[ni < (uint32_t)GLIST ? ni : (uint32_t)GLIST - 1u];
      one(check_v, e, b < cnt);
    }
#endif
  };

  // Compact table clear and flush (few active words, no churn): the nf <= 32 active words of
  // the slice are ranked (rank = position in the packed E row) and lane l serves rank
  // l % seg of connection l / seg, so one LDS / store / atomic instruction covers 64 / seg
  // connections instead of one (light dense rounds: ~8 active words, 4 connections at once).
  // The picks touch only the active words' table columns, so only those are cleared.
  const int nf = __popcll(fam);
  const bool compact = P2PG_COMPACT && !CHURN && anyf && nf <= 32 &&
                       (STORE_E ? st.AW[cur] != nullptr : g.gone == nullptr);
  const bool use_tbl = anyf && !all;
  int seg = 64, rk_lane = 0, wc = 0, gl = 0;
  bool rk = false;
  if (compact) {
    seg = nf <= 16 ? 16 : 32;
    const int rank = (int)__builtin_amdgcn_mbcnt_hi(
        (uint32_t)(fam >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fam, 0u));
    // every active word pushes its index to lane `rank`; the others to lane 63 (never read)
    const int wr = __builtin_amdgcn_ds_permute((f ? rank : 63) << 2, lane);
    rk_lane = lane & (seg - 1);
    wc = __builtin_amdgcn_ds_bpermute(rk_lane << 2, wr);  // the word of rank rk_lane
    rk = rk_lane < nf;
    gl = lane / seg;
  }
  const int gper = 64 / seg;

  if (PH != 2 && use_tbl) {
    if (compact) {
      for (int j0 = 0; j0 < nn; j0 += gper) {
        const int jj = j0 + gl;
        if (rk && jj < nn) tbl_clear(L, jj, wc);
      }
    } else {
      for (int j = 0; j < nn; ++j) {
        tbl_clear(L, j, lane);
      }
    }
    const uint32_t cnt = (uint32_t)__popcll(f);
    // at most one new bit per word (light rounds: ~9 bits in ~8 words per peer): lane w's word
    // is its own entry, one Philox batch with no list (the scan, the list writes and a sync cost
    // more than the batch itself there)
    bool direct = false;
    if constexpr (DIRECT && K > 0 && P2PG_PICK_DIRECT) {
      direct = __ballot(cnt > 1u) == 0ull;
      if (direct) {
        wave_lds_sync();  // (the table clear above, before the table atomics)
        const uint32_t e = ((uint32_t)lane << 6) | (uint32_t)__builtin_ctzll(f | (1ull << 63));
        if (nb == 0 && nn == (int)deg)
          one(std::false_type{}, e, f != 0ull);
        else
          one(std::true_type{}, e, f != 0ull);
        wave_lds_sync();
        PROF_MARK(7);
      }
    }
    // word-major compaction: lane w lists its word's set bits at its exclusive prefix-sum
    // position (one DPP scan; a 32-bit ctz / clear per bit), so every lane gets an equal
    // share of the Philox work; pick_batch reads the list strided (distinct words per batch)
    const uint32_t incl = direct ? 0u : wave_scan_u32(cnt);
    const uint32_t total = direct ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t pos0 = incl - cnt;
    // a pass lists GLIST - 1 entries; the last list slot takes the entries not written
    constexpr uint32_t CAP = (uint32_t)GLIST - 1u;
    for (uint32_t lb = 0; lb < total; lb += CAP) {
      const uint32_t nw = total - lb < CAP ? total - lb : CAP;
      list_bits(L.lst, CAP, f, (uint32_t)lane << 6, pos0 - lb, nw);
      wave_lds_sync();
      PROF_MARK(6);
      const uint32_t n = nw;
      if constexpr (K > 0) {
        // a source whose whole adjacency is this chunk needs no range check on its picks
        if (nb == 0 && nn == (int)deg)
          pick_batch(std::false_type{}, n);
        else
          pick_batch(std::true_type{}, n);
      } else {
        for (uint32_t i = lane; i < n; i += 64) {
          const uint32_t e = L.lst[i];
          const uint32_t wl = e >> 6, bit = e & 63u;
          const uint32_t mg = p.msg_base + (uint32_t)((sl * 64 + (int)wl) * 64) + bit;
          uint32_t* const col = &L.tbl[tbl_ix(0u, wl, bit >> 5)];
          const uint32_t mb = 1u << (bit & 31u);
          uint32_t pk[16];
          gossip_picks((uint32_t)p.round, gv, mg, (uint32_t)deg, k, p.gseed_lo, p.gseed_hi, pk);
          for (int q = 0; q < k; ++q) {
            const uint32_t jj = pk[q] - (uint32_t)nb;
            if (jj < (uint32_t)nn) atomicOr(col + jj * 128u, mb);
          }
        }
      }
      wave_lds_sync();
      PROF_MARK(7);
    }
  }
  if constexpr (PH == 1) return;
  if (compact) {
    const uint64_t segm = (1ull << seg) - 1ull;
    uint64_t fr = 0;
    if (all) {
      const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(wc << 2, (int)(uint32_t)f);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(wc << 2, (int)(uint32_t)(f >> 32));
      fr = ((uint64_t)hi << 32) | lo;
    }
    for (int j0 = 0; j0 < nn; j0 += gper) {
      const int jj = j0 + gl;
      const bool ok = rk && jj < nn;
      uint64_t x = 0;
      if (ok) x = all ? fr : tbl_word(L, jj, wc);
      const uint32_t nj = (uint32_t)__builtin_amdgcn_ds_bpermute(
          (nbr0 + (jj < nn ? jj : 0)) << 2, (int)nbr);
      const uint64_t bal = __ballot(ok && x != 0ull);
      if (STORE_E && !(PART && (nj & REV_GHOST))) {
        if (ok) st_row(at_row(Eo, nj, W) + rk_lane, x);
      } else {
        const int64_t u = (int64_t)(PART ? nj & ~REV_GHOST : nj);
        if (x) atomicOr((unsigned long long*)at_row(nx, u, W) + sl * 64 + wc, (unsigned long long)x);
        if (rk_lane == 0 && ((bal >> (lane & ~(seg - 1))) & segm))
          atomicOr(&Tn[u >> 5], 1u << (u & 31));
      }
      if (lane == 0) c[ST_SCATTER] += (CT)__popcll(bal);
    }
    PROF_MARK(8);
    return;
  }
  auto tbl_row = [&](int j) -> uint64_t {
    return tbl_word(L, j, lane);
  };
  uint64_t xn = use_tbl && nn > 0 ? tbl_row(0) : 0ull;
  for (int j = 0; j < nn; ++j) {
    const uint64_t x = all ? f : xn;  // row j; row j + 1 is read before row j is stored
    if (use_tbl && j + 1 < nn) xn = tbl_row(j + 1);
    const uint64_t bal = __ballot(x != 0ull);
    const uint32_t nj = (uint32_t)__builtin_amdgcn_readlane((int)nbr, nbr0 + j);
    if (STORE_E) {
      bool dropped = false;
      if (CHURN && bal)
        dropped = churn_dropped((uint32_t)p.round, gv, gidx_s(g, ldc(g.colidx + rb + nb + j)),
                                p.churn_thr, p.cseed_lo, p.cseed_hi);
      if (PART && (nj & REV_GHOST)) {  // a ghost's connection: its row push, exchanged
        const int64_t u = (int64_t)(nj & ~REV_GHOST);
        if (!dropped && bal) {
          if (x) atomicOr((unsigned long long*)at_row(nx, u, W) + w, (unsigned long long)x);
          if (lane == 0) {
            atomicOr(&Tn[u >> 5], 1u << (u & 31));
            c[ST_SCATTER] += (CT)__popcll(bal);
          }
        }
        continue;
      }
      // receiver-major: the row lands in the RECEIVER's slot for this connection, so the
      // pull streams its own contiguous slot range; packed: only the active words, in order
      if (st.AW[cur]) {
        if (f) st_row(at_row(Eo, nj, W) + __popcll(fam & ((1ull << lane) - 1ull)), dropped ? 0ull : x);
      } else if (valid) {
        st_row(at_row(Eo, nj, W) + w, dropped ? 0ull : x);
      }
      if (!dropped && lane == 0) c[ST_SCATTER] += (CT)__popcll(bal);
    } else {
      if (!bal) continue;
      if (g.gone && g.gone[rb + nb + j]) continue;  // connection removed: the push is lost
      const int64_t u = (int64_t)nj;
      if (CHURN && churn_dropped((uint32_t)p.round, gv, gidx_s(g, u), p.churn_thr,
                                 p.cseed_lo, p.cseed_hi))
        continue;
      if (x) atomicOr((unsigned long long*)at_row(nx, u, W) + w, (unsigned long long)x);
      if (lane == 0) {
        atomicOr(&Tn[u >> 5], 1u << (u & 31));
        c[ST_SCATTER] += (CT)__popcll(bal);
      }
    }
  }
  PROF_MARK(8);
}

// The scatter launch: tasks [task0, nwords) are 32-peer bitmap words (sources with deg <=
// GCHUNK), tasks from nwords on are groups of 64 (wide source, chunk) items.  task0 = nwords
// runs the items only (fused rounds: the items of the pull hubs, deg > HUB_T).
template <bool CHURN, int K, bool STORE_E, bool PART = false>
__global__ __launch_bounds__(256) void k_gossip_scatter(DevGraph g, DevState st, RoundParams p,
                                                        const int64_t* __restrict__ hub_items,
                                                        int64_t n_hub, int64_t task0) {
  __shared__ ScatterLds lds[WPB];
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  ScatterLds& L = lds[wib];
  const int64_t V = g.V;
  const int W = st.W;
  const int cur = p.round & 1;
  const uint64_t* __restrict__ Fc = st.F[cur];
  // packed rows: a frontier word counts only under the row's AW mask (an update that ran with
  // RoundParams::store_f == 2 leaves stale words outside it)
  const uint64_t* __restrict__ AWc = W <= 64 ? st.AW[cur] : nullptr;
  const int64_t nwords = (V + 31) >> 5;
  const int64_t ntasks = nwords + ((n_hub + 63) >> 6);
  const int nslices = (W + 63) >> 6;
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};
  PROF_DECL  // development builds: segment clocks of this kernel are not reported

  // lane j's neighbour datum for the chunk starting at slot rb + nb
  auto load_nbr = [&](int64_t rb, int nn) -> uint32_t {
    if (lane >= nn) return 0u;
    return STORE_E ? g.rev[rb + lane] : (uint32_t)g.colidx[rb + lane];
  };

  // one 32-peer bitmap task of single-slice rows (W <= 64), pipelined: row offsets of the
  // peers by scalar loads; the next active peer's frontier word and receiver slots are in
  // flight while the current one computes
  auto bitmap_task = [&](int64_t task, uint32_t todo) {
      const int64_t base = task << 5;
      // row offsets by SCALAR loads (lgkmcnt): a vector load here would make every vertex
      // wait on vmcnt, i.e. on the previous vertex's outstanding row stores
      auto pick_next = [&](uint32_t& t, int64_t& rb, int64_t& deg) -> int {
        while (t) {
          const int b = __builtin_ctz(t);
          t &= t - 1u;
          const int64_t vv = __builtin_amdgcn_readfirstlane((int)(base + b));
          rb = ldc(g.rowptr + vv);
          deg = ldc(g.rowptr + vv + 1) - rb;
          if (deg <= GCHUNK) return b;  // wider sources: their chunk items
        }
        return -1;
      };
      int64_t rb1 = 0, deg1 = 0, rb2 = 0, deg2 = 0;
      int b1 = pick_next(todo, rb1, deg1);
      uint64_t f1 = 0;
      uint32_t rv1 = 0;
      if (b1 >= 0) {
        if (lane < W && aw_has(AWc, base + b1, lane)) f1 = Fc[(base + b1) * W + lane];
        rv1 = load_nbr(rb1, (int)deg1);
      }
      while (b1 >= 0) {
        const int b2 = pick_next(todo, rb2, deg2);
        uint64_t f2 = 0;
        uint32_t rv2 = 0;
        if (b2 >= 0) {
          if (lane < W && aw_has(AWc, base + b2, lane)) f2 = Fc[(base + b2) * W + lane];
          rv2 = load_nbr(rb2, (int)deg2);
        }
        scatter_row<CHURN, K, STORE_E, 0, PART>(g, st, p, L, lane, base + b1, rb1, deg1, 0, 0, f1, rv1, 0,
                                       c PROF_PASS);
        b1 = b2;
        rb1 = rb2;
        deg1 = deg2;
        f1 = f2;
        rv1 = rv2;
      }
  };
  int64_t first = task0;
  if (nslices == 1 && task0 < nwords) {
    // SCAN_W activity words per wave pass (lane = task): the active tasks of a sparse round
    // are found with one load per lane instead of one dependent load per task
    const int64_t wave = (int64_t)blockIdx.x * WPB + wib, nwave = (int64_t)gridDim.x * WPB;
    for (int64_t tb = task0 + wave * SCAN_W; tb < nwords; tb += nwave * SCAN_W) {
      const int64_t tl = tb + lane;
      const uint32_t al = lane < SCAN_W && tl < nwords ? st.A[cur][tl] : 0u;
      uint64_t busy = __ballot(al != 0u);
      while (busy) {
        const int l = __builtin_ctzll(busy);
        busy &= busy - 1ull;
        bitmap_task(tb + l, (uint32_t)__builtin_amdgcn_readlane((int)al, l));
      }
    }
    first = nwords;
  }
  for (int64_t task = first + (int64_t)blockIdx.x * WPB + wib; task < ntasks;
       task += (int64_t)gridDim.x * WPB) {
    auto one_source = [&](int64_t v, int chunk) {
      const int64_t rb = g.rowptr[v];
      const int64_t deg = g.rowptr[v + 1] - rb;
      const int nb = chunk * GCHUNK;
      const int nn = (int)(deg - nb < GCHUNK ? deg - nb : GCHUNK);
      const uint32_t rv = load_nbr(rb + nb, nn);
      for (int sl = 0; sl < nslices; ++sl) {
        const int w = sl * 64 + lane;
        const uint64_t f = w < W && aw_has(AWc, v, w) ? Fc[v * W + w] : 0ull;
        scatter_row<CHURN, K, STORE_E, 0, PART>(g, st, p, L, lane, v, rb, deg, chunk, sl, f, rv, 0, c PROF_PASS);
      }
    };
    if (task < nwords) {  // multi-slice rows (W > 64)
      uint32_t todo = st.A[cur][task];
      while (todo) {
        const int b = __builtin_ctz(todo);
        todo &= todo - 1u;
        const int64_t v = (task << 5) + b;
        if (g.rowptr[v + 1] - g.rowptr[v] > GCHUNK) continue;  // wide: its chunk items
        one_source(v, 0);
      }
      continue;
    }
    // 64 (wide source, chunk) items per task, their activity tested lane-parallel: in sparse
    // rounds almost every item is skipped, and one dependent load chain per item would make
    // an idle launch cost ~0.3 ms (config 4 has ~1.4M items)
    const int64_t i = (task - nwords) * 64 + lane;
    int64_t item = 0;
    bool act = false;
    if (i < n_hub) {
      item = hub_items[i];
      act = bit_test(st.A[cur], item >> 32);
    }
    uint64_t am = __ballot(act);
    while (am) {
      const int l = __builtin_ctzll(am);
      am &= am - 1ull;
      const int64_t it = readlane64(item, l);
      one_source(it >> 32, (int)(it & 0xFFFFFFFFll));
    }
  }
  flush_stats(st.stats, c, lane);
}

// Active neighbours whose E words the fused kernel keeps in flight across a target's picks.
#ifndef P2PG_FG
#define P2PG_FG 8
#endif
constexpr int FG = P2PG_FG;



// Gossip dense round r >= 1 after a dense round r-1: the pull of round r (k_pull1<false,
// true>: arrivals = packed E[(r-1)&1] rows of the active neighbours) and, for every peer with
// a first receipt, its own round-r pushes (scatter_row<STORE_E> into E[r&1]) in the same
// pass.  The new frontier row goes straight from registers into the picks (no HBM round trip,
// no second pass over the peers), and the Philox work of one target overlaps the first
// gathers of the next target, which are already in flight.  Hubs (deg > HUB_T) are pulled by k_pull_hub_*
// and pushed by a chunk-item scatter launch over the hubs only.
// Waves per SIMD the launch bounds ask for.  Both 3 and 4 compile to under 128 VGPRs (W = 64:
// 118 vs 114, no VGPR spills, ~160 SGPRs spilled to VGPR lanes either way), so 4 waves stay
// resident per SIMD; the looser bound only changes the compiler's schedule, which measured
// 1.3-1.4 ms per c4 step faster on two boxes (2: no better; W = 32 / 16 shares equal,
// profiles/r04/ab_fused_waves.txt)
#ifndef P2PG_FUSED_WAVES
#define P2PG_FUSED_WAVES 3
#endif
// MODE 0: the fused dense round above.
// MODE 1, PO (push only): the first dense round after an update (16 < W <= 64, packed E) -- the
// peers are the round's active non-hub peers, their arrivals are their own frontier rows F[r&1]
// (dedup, counters, bitmaps and AW were done by the update), and only the picks and the E stores
// run, through the same software pipeline (replaces k_gossip_scatter<.., true>: one wave per
// source with a two-deep prefetch, ~7.3 ms per c4 step at W = 64 and at W = 32).
// MODE 2, UP (update + push): the same first dense round with the update folded in -- the peers
// are the touched non-hub peers (T[r&1]), their arrivals the row pushes next[r&1] of the sparse
// round before (read and cleared), then dedup, frontier row, bitmaps, counters and the pushes as
// in a fused round; the touched hubs are left in T for a hub-only update (launch_gossip_update_push).
// MODE 3, PL (pull only): the last dense round before the sparse ones (32 < W <= 64) -- arrivals,
// dedup, frontier rows and bitmaps as in MODE 0, no picks and no E stores (the round's pushes go by
// row atomics afterwards); the software pipeline runs across task boundaries, which k_pull1's
// per-task three-stage pipeline does not.
// HALF (MODE 0, W <= 32): arrivals gathered two slots per load (src_word_pair).
// PART (vertex-partitioned gossip ranks, 16 < W <= 64): no E slot of a ghost neighbour is gathered
// (REV_GHOST in rev; its sends arrive as exchanged row pushes, next[r&1] + T bits, ORed into the
// arrivals here), pushes to ghosts go to their row pushes (scatter_row PART), Philox ids are
// global (gid).  The caller clears the consumed row pushes afterwards (launch_clear_arrivals).
template <bool CHURN, int K, int MODE = 0, bool HALF = false, bool PART = false>
__global__ __launch_bounds__(256, P2PG_FUSED_WAVES) void k_gossip_fused(DevGraph g, DevState st,
                                                                        RoundParams p) {
  constexpr bool PO = MODE == 1, UP = MODE == 2, PL = MODE == 3;
  constexpr bool GATHER = MODE == 0 || PL;  // arrivals gathered from E
  static_assert(!(PART && UP), "no update+push pass on partitioned ranks");
  // (not partitioned: local ids are the Philox ids) and never on a pre-update graph: known here,
  // so the id translation and lost-slot tests fold away (fewer live scalar registers)
  if (!PART) g.gid = nullptr;
  g.gone = nullptr;
  g.gdeg = g.gpos = nullptr;
  __shared__ ScatterLds lds[WPB];
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int64_t V = g.V;
  const int W = st.W;
  const int cur = p.round & 1, prv = cur ^ 1;
  const uint64_t* __restrict__ Src = st.E[prv];
  uint64_t* __restrict__ Fc = st.F[cur];
  const uint32_t* __restrict__ Ap = st.A[prv];
  const uint64_t* __restrict__ AWp = st.AW[prv];
  const int64_t ntasks = (V + 31) >> 5;
  const bool valid = lane < W;
  const uint64_t fm = valid ? full_mask(lane, W, st.M) : 0ull;
  // per-lane counters are 32-bit and per task (<= 32 peers, none a hub: no overflow), folded
  // into wave-uniform 64-bit totals after each task (fewer live VGPRs than 64-bit lanes)
  // wave totals in 32 bits (8 fewer scalar registers): balanced_grid never gives a wave more
  // than TASKS_PER_WAVE_MAX tasks, which keeps its relay / wedge sums (<= tasks x 32 peers x 4096
  // messages x fanout 16; hubs excluded) below 2^32 (c4: ~2.4 tasks per wave)
  uint32_t tot[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};
  PROF_DECL

  // Issuer (wave-uniform): this wave's tasks in grid-stride order and, in each, its
  // unsaturated non-hub peers in ascending order.  The next task's saturated / hub words and
  // row offsets are loaded while the current one is issued, so the software pipeline below runs
  // straight across task boundaries (restarting it per 32-peer task cost 3-4 dependent memory
  // trips: ~12 % of a light round).
  const int64_t tstride = (int64_t)gridDim.x * WPB;
  int64_t pf_task = (int64_t)blockIdx.x * WPB + wib;  // prefetched task (-1: none left)
  uint32_t pf_s = 0, pf_h = 0;
  uint32_t pf_rp = 0;  // slot offsets fit 32 bits (rev[] holds slot ids as uint32)
  auto prefetch = [&](int64_t t) {
    pf_task = t;
    if (t < 0) return;
    // PO: the active peers; UP: the touched ones; else the saturated ones
    pf_s = PO ? st.A[cur][t] : UP ? st.T[cur][t] : st.S[t];
    pf_h = g.H ? g.H[t] : 0u;
    const int64_t u0 = t << 5;
    pf_rp = (lane <= 32 && u0 + lane <= V) ? (uint32_t)g.rowptr[u0 + lane] : 0u;
  };
  if (pf_task >= ntasks) pf_task = -1;
  prefetch(pf_task);
  int32_t it_u0 = 0;     // first peer of the issuing task
  uint32_t it_rest = 0;  // its peers not issued yet
  uint32_t rp = 0;       // lane l <= 32: rowptr[it_u0 + l]
  // next peer to issue (global id; -1 when this wave's tasks are done) and its slot range
  auto next_peer = [&](uint32_t& beg, uint32_t& end) -> int32_t {
    while (!it_rest) {
      const int64_t t = pf_task;
      if (t < 0) return -1;
      const int64_t u0 = t << 5;
      const uint32_t sw = (uint32_t)__builtin_amdgcn_readfirstlane((int)pf_s);
      const uint32_t hw = (uint32_t)__builtin_amdgcn_readfirstlane((int)pf_h);
      uint32_t todo = (PO || UP ? sw : ~sw) & ~hw;
      if (V - u0 < 32) todo &= (1u << (V - u0)) - 1u;
      // UP: the non-hub touched peers are consumed here (only this wave reads this T word)
      if (UP && lane == 0 && (sw & ~hw)) st.T[cur][t] = sw & hw;
      rp = pf_rp;
      prefetch(t + tstride < ntasks ? t + tstride : -1);
      if (!todo) {
        if (!PO && lane == 0) st.A[cur][t] = 0u;
        continue;
      }
      it_u0 = (int32_t)u0;
      it_rest = todo;
    }
    const int b = __builtin_ctz(it_rest);
    it_rest &= it_rest - 1u;
    beg = (uint32_t)__builtin_amdgcn_readlane((int)rp, b);
    end = (uint32_t)__builtin_amdgcn_readlane((int)rp, b + 1);
    return it_u0 + b;
  };

  auto issue = [&](FusedStage& q) {
    q.v = 0;
    q.rv = 0;
    q.s = 0;
    q.u = next_peer(q.beg, q.end);
    if (q.u < 0) return;
    // PO: the peer's frontier row (its new receipts of this round) instead of its seen row;
    // UP: the seen row and, in the stage's mask field, the push row (the arrivals)
    if (valid) q.s = ld_once(at_row(PO ? Fc : st.seen, q.u, W) + lane);
    if (UP) q.am = valid ? at_row(st.next[cur], q.u, W)[lane] : 0ull;
    // PO: the row's active-word mask (a frontier row written by the update may hold stale words
    // outside it, RoundParams::store_f == 2)
    if (PO) q.am = ldc(st.AW[cur] + q.u);
    const uint32_t j = q.beg + lane;
    if (j < q.end) {
      if (GATHER) q.v = ld_once(&g.colidx[j]);
      if (!PL || PART) q.rv = ld_once(&g.rev[j]);  // (PART: ghost marks)
    }
  };
  // loads only; gather() tests the bit (see k_pull1)
  auto activity = [&](FusedStage& q) {
    if (!GATHER || q.u < 0) return;
    const uint32_t j = q.beg + lane;
    q.am = 0;
    q.aword = 0;
    if (j < q.end) {
      q.am = AWp[q.v];
      q.aword = Ap[q.v >> 5];
    }
  };

  // the first FG active neighbours' words of q go out into X; mr = q's active slots (of its
  // first 64) still to gather
  uint64_t X[FG];
  auto gather = [&](const FusedStage& q, uint64_t& mr) {
    if (!GATHER) {  // no arrivals to gather: they came with the row stage
#pragma unroll
      for (int k = 0; k < FG; ++k) X[k] = 0ull;
      mr = 0;
      return;
    }
    const uint64_t needm = __ballot((fm & ~q.s) != 0ull);
    const uint32_t jq = q.beg + lane;
    uint64_t m = __ballot(jq < q.end && ((q.aword >> (q.v & 31)) & 1u) &&
                          !(PART && (q.rv & REV_GHOST)));
    if constexpr (HALF) {  // FG slots in flight, two per load (FG / 2 loads)
      constexpr int FH = FG / 2;
      uint32_t r0[FH], r1[FH], m0[FH], m1[FH];
#pragma unroll
      for (int k = FH; k < FG; ++k) X[k] = 0ull;
#pragma unroll
      for (int k = 0; k < FH; ++k) {
        r0[k] = r1[k] = m0[k] = m1[k] = 0u;
        if (m) {
          const int i0 = __builtin_ctzll(m);
          m &= ~(1ull << i0);
          r0[k] = q.beg + (uint32_t)i0;
          m0[k] = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)q.am, i0);
        }
        if (m) {
          const int i1 = __builtin_ctzll(m);
          m &= ~(1ull << i1);
          r1[k] = q.beg + (uint32_t)i1;
          m1[k] = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)q.am, i1);
        }
      }
#pragma unroll
      for (int k = 0; k < FH; ++k)
        X[k] = src_word_pair(Src, r0[k], r1[k], W, m0[k], m1[k], m0[k] & (uint32_t)needm,
                             m1[k] & (uint32_t)needm);
      mr = m;
      return;
    }
    // all slot ids / word masks first, then all FG loads back to back: a readlane between
    // two loads would make the wave wait for the first one (merged vmcnt state)
    // (a slot past the last active one keeps am = 0: its load mask is empty, no select needed)
    uint32_t sv[FG];
    uint64_t am[FG];
#pragma unroll
    for (int k = 0; k < FG; ++k) {
      sv[k] = 0u;
      am[k] = 0ull;
      if (m) {
        const int idx = __builtin_ctzll(m);
        m &= ~(1ull << idx);
        sv[k] = q.beg + (uint32_t)idx;  // receiver-major E: the row of slot j is j
        am[k] = (uint64_t)readlane64((int64_t)q.am, idx);
      }
    }
#pragma unroll
    for (int k = 0; k < FG; ++k) X[k] = src_word_m(Src, sv[k], W, am[k], am[k] & needm);
    mr = m;
  };

  // Per consumed task: activity word, newly saturated peers and the per-lane counters (32-bit,
  // <= 32 peers per fold, none a hub: no overflow), folded into wave-uniform 64-bit totals when
  // the consumer moves on to the next task.
  uint32_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t ct = -1;
  uint32_t aw = 0, nsat = 0;
  auto finish_task = [&]() {
    if (ct < 0) return;
    if (!PO && lane == 0) {  // PO: the update wrote the task's bitmaps
      st.A[cur][ct] = aw;
      if (nsat) atomicOr(&st.S[ct], nsat);  // this wave owns the task: no other writer
    }
#pragma unroll
    for (int q = 0; q < STAT_N; ++q) {
      if (q == ST_ACTIVE_V) continue;
      const uint32_t r = wave_reduce_u32<false>(c[q]);
      c[q] = 0;
      if (q == ST_ACTIVE_W) {
        // one register for two per-task counts (each <= 64 lanes x 32 peers < 2^16): active
        // words in the low half, active peers (lane 0) in the high half
        tot[ST_ACTIVE_W] += r & 0xFFFFu;
        tot[ST_ACTIVE_V] += r >> 16;
      } else {
        tot[q] += r;
      }
    }
    aw = 0;
    nsat = 0;
  };

  // Software pipeline, per target t: rows L2(t+3) -> activity L3(t+2) -> gathers(t+1) ->
  // consume(t).  The first gathers of target t+1 are issued BEFORE target t's stores and
  // picks, so their latency hides behind t's Philox / LDS work.  The four stages rotate by
  // unrolling (step(A,B,C,D), step(B,C,D,A), ...), never by copying: a register copy of a
  // load still in flight would make the wave wait for it (and, vmcnt being in order, for
  // every younger load and store) at the end of each target.
  // The flush (E stores) of a short row (deg <= GCHUNK) is deferred to the next target,
  // after that target's gather wait: a wait issued right behind a row's stores would also
  // wait for their completion (vmcnt counts loads and stores in order); one target later,
  // the picks in between have covered it.
  bool pend = false;
  int64_t pu = 0, pbeg = 0, pdeg = 0;
  uint64_t pnw = 0;
  uint32_t prcv = 0;  // its receiver slots
  auto flush_pending = [&]() {
    if (pend) {
      scatter_row<CHURN, K, true, 2, PART>(g, st, p, lds[wib], lane, pu, pbeg, pdeg, 0, 0, pnw, prcv,
                                     0, c PROF_PASS);
      pend = false;
    }
  };
  FusedStage sA, sB, sC, sD;
  issue(sA);
  issue(sB);
  activity(sA);
  if (sA.u >= 0) gather(sA, sA.mr);
  activity(sB);
  issue(sC);
  PROF_MARK(5);

  // consume a (gathers in X), advance b (gathers), c (activity), d (rows), then a's picks
  auto step = [&](FusedStage& a, FusedStage& b, FusedStage& cc, FusedStage& d) {
    const int64_t u = a.u;
    if ((u >> 5) != ct) {
      finish_task();
      ct = u >> 5;
    }
    const uint64_t deg = (uint64_t)(a.end - a.beg);
    const uint64_t need = PO ? ~0ull : fm & ~a.s;
    const uint64_t needm = __ballot(need != 0ull);
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < FG; ++k) acc |= X[k];
    if (UP) acc = a.am;  // the push row
    // PART: the rows other ranks pushed to u in the last round (exchanged; T bit), loaded now so
    // the wait below covers them
    uint64_t remote = 0;
    if (PART && GATHER && ((ldc(st.T[cur] + (u >> 5)) >> (u & 31)) & 1u) && valid)
      remote = ld_once(at_row(st.next[cur], u, W) + lane);
    PROF_MARK(0);
    if (GATHER) {
      uint64_t m = a.mr;  // the rest of the first 64 slots, then further 64-slot chunks
      uint64_t sam = a.am;
      uint32_t cb = a.beg;
      for (;;) {
        while (HALF && m) {  // 8 slots per trip, two per load
          uint32_t r0[4], r1[4], m0[4], m1[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            r0[k] = r1[k] = m0[k] = m1[k] = 0u;
            if (m) {
              const int i0 = __builtin_ctzll(m);
              m &= ~(1ull << i0);
              r0[k] = cb + (uint32_t)i0;
              m0[k] = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sam, i0);
            }
            if (m) {
              const int i1 = __builtin_ctzll(m);
              m &= ~(1ull << i1);
              r1[k] = cb + (uint32_t)i1;
              m1[k] = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sam, i1);
            }
          }
          uint64_t x[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            x[k] = src_word_pair(Src, r0[k], r1[k], W, m0[k], m1[k], m0[k] & (uint32_t)needm,
                                 m1[k] & (uint32_t)needm);
#pragma unroll
          for (int k = 0; k < 4; ++k) acc |= x[k];
        }
        while (!HALF && m) {
          uint32_t sv[8];
          uint64_t am[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            am[k] = 0ull;  // (past the last active slot: an empty load mask)
            if (m) {
              const int idx = __builtin_ctzll(m);
              m &= ~(1ull << idx);
              sv[k] = cb + (uint32_t)idx;  // the E row of slot cb + idx (receiver-major)
              am[k] = (uint64_t)readlane64((int64_t)sam, idx);
            } else {
              sv[k] = 0u;
            }
          }
          uint64_t x[8];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            x[k] = src_word_m(Src, sv[k], W, am[k], am[k] & needm);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc |= x[k];
        }
        cb += 64;
        if (cb >= a.end) break;
        const uint32_t j = cb + lane;  // further chunks of a wide row: serial
        bool act = false;
        sam = 0;
        if (j < a.end) {
          const int32_t v = g.colidx[j];
          act = bit_test(Ap, v) && !(PART && (g.rev[j] & REV_GHOST));
          if (act) sam = AWp[v];
        }
        m = __ballot(act);
      }
    }
    // Everything loaded before this point (this target's rows, the next target's activity
    // words, the prefetched task words) has landed or is about to: wait for it explicitly
    // HERE, so that the compiler knows it has arrived and inserts no vmcnt wait behind the next
    // target's gathers when this target's row words are used below (vmcnt is in order: such a
    // wait would stall until those gathers return).
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    PROF_MARK(1);
    if (HALF) acc |= bperm64(lane ^ 32, acc);  // lanes 32-63 gathered for words 0-31 too
    if (PART) acc |= remote;
    if (UP && acc) {  // the push row is consumed: all-zero again outside touched rows
      st_prow(at_row(st.next[cur], u, W) + lane, 0ull);
      c[ST_AUX] += 1;  // touched (pushed-to) words consumed
    }
    flush_pending();
    // advance the pipeline before this target's stores and picks: gathers of t+1 (their
    // activity words were loaded a target ago), activity words of t+2, rows of t+3
    if (b.u >= 0) gather(b, b.mr);
    activity(cc);
    issue(d);
    PROF_MARK(2);
    const uint64_t nw = PO ? ((a.am >> lane) & 1ull ? a.s : 0ull) : acc & need;
    const uint64_t wm = __ballot(nw != 0ull);
    if (!PO && nw) {
      st_frow(at_row(st.seen, u, W) + lane, a.s | nw);
      const uint32_t pc = (uint32_t)__popcll(nw);
      const uint32_t kf = K > 0 ? (uint32_t)K : (uint32_t)p.fanout;
      const uint32_t per_bit = deg < (uint64_t)kf ? (uint32_t)deg : kf;
      c[ST_NEW] += pc;
      c[ST_RELAYS] += pc * per_bit;
      c[ST_ACTIVE_W] += 1;
      c[ST_WEDGES] += (uint32_t)deg;
    }
    if (wm) {
      if (!PO) {
        if (valid && p.store_f && (p.store_f != 2 || nw)) st_frow(at_row(Fc, u, W) + lane, nw);
        aw |= 1u << (u & 31);
        if (lane == 0) {
          st.AW[cur][u] = wm;
          c[ST_ACTIVE_W] += 1u << 16;  // ST_ACTIVE_V, packed (see finish_task)
          c[ST_DEG_ACT] += (uint32_t)deg;
        }
      }
      // this round's pushes, GCHUNK connections at a time.  a.rv holds the receiver slots of
      // the first 64 (arrived: see the explicit wait above); wider rows load the next 64
      // every 4 chunks and wait for them right there -- a load that MAY be in flight when
      // the picks read the slots would make the compiler wait for everything, the next
      // target's gathers included.
      if (PL) {
        // (no pushes: the sparse push that follows reads the frontier row)
      } else if (deg <= (uint64_t)GCHUNK) {
        scatter_row<CHURN, K, true, 1, PART, PO || UP>(g, st, p, lds[wib], lane, u, a.beg, (int64_t)deg, 0, 0,
                                       nw, a.rv, 0, c PROF_PASS);
        pend = true;
        pu = u;
        pbeg = a.beg;
        pdeg = (int64_t)deg;
        pnw = nw;
        prcv = a.rv;
      } else if (deg <= 64) {
        for (int ch = 0; (int64_t)ch * GCHUNK < (int64_t)deg; ++ch)
          scatter_row<CHURN, K, true, 0, PART, PO || UP>(g, st, p, lds[wib], lane, u, a.beg, (int64_t)deg, ch, 0,
                                      nw, a.rv, ch * GCHUNK, c PROF_PASS);
      } else {
        for (int ch = 0; (int64_t)ch * GCHUNK < (int64_t)deg; ++ch) {
          const int off = (ch * GCHUNK) & 63;
          const uint32_t j = a.beg + (uint32_t)(ch * GCHUNK - off) + lane;
          const uint32_t rvb = j < a.end ? g.rev[j] : 0u;
          __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
          scatter_row<CHURN, K, true, 0, PART, PO || UP>(g, st, p, lds[wib], lane, u, a.beg, (int64_t)deg, ch, 0,
                                      nw, rvb, off, c PROF_PASS);
        }
      }
    }
    PROF_MARK(3);
    if (!PO && !__ballot(valid && (a.s | nw) != fm)) nsat |= 1u << (u & 31);
  };
  for (;;) {
    if (sA.u < 0) break;
    step(sA, sB, sC, sD);
    if (sB.u < 0) break;
    step(sB, sC, sD, sA);
    if (sC.u < 0) break;
    step(sC, sD, sA, sB);
    if (sD.u < 0) break;
    step(sD, sA, sB, sC);
  }
  flush_pending();
  finish_task();
  PROF_MARK(4);
  PROF_FLUSH
  if (lane == 0) {
    unsigned long long* shard = st.stats + (blockIdx.x & (STAT_SHARDS - 1)) * STAT_N;
#pragma unroll
    for (int q = 0; q < STAT_N; ++q)
      if (tot[q]) atomicAdd(shard + q, (unsigned long long)tot[q]);
  }
}

// ---------------------------------------------------------------------------------------
// Validation: the lowest-id neighbour v whose round-(r-1) send of message m reached u
// (receivers process senders in ascending id -- the harness's stand-in for TCP arrival
// order).  Returns -2 if none (cannot happen for a first receipt at r >= 1).
__device__ int32_t find_parent(const DevGraph& g, const DevState& st, const RoundParams& p,
                               int64_t u, int m) {
  const int prv = (p.round & 1) ^ 1;
  const int W = st.W;
  const uint64_t bit = 1ull << (m & 63);
  const int w = m >> 6;
  const int64_t beg = g.rowptr[u], end = g.rowptr[u + 1];
  for (int64_t e = beg; e < end; ++e) {
    const int32_t v = g.colidx[e];
    if (g.gone && g.gone[e]) continue;  // lost with its connection (topology update)
    if (!bit_test(st.A[prv], v)) continue;
    if (!(st.F[prv][(int64_t)v * W + w] & bit)) continue;
    if (p.churn_thr && churn_dropped((uint32_t)(p.round - 1), gidx(g, u), gidx(g, v),
                                     p.churn_thr, p.cseed_lo, p.cseed_hi))
      continue;
    if (p.mode == 1) {
      const int64_t vb = g.rowptr[v];
      // a ghost sender (partitioned runs): its global degree and u's place in its global row
      const bool ghost = g.gpos && g.gpos[e] >= 0;
      const int64_t dv = ghost ? (int64_t)g.gdeg[v] : g.rowptr[v + 1] - vb;
      if (dv > p.fanout) {
        int64_t lo = 0, hi = dv;  // position of u in v's ascending list
        if (ghost) {
          lo = g.gpos[e];
        } else {
          while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (g.colidx[vb + mid] < u) lo = mid + 1; else hi = mid;
          }
        }
        uint32_t pk[16];
        gossip_picks((uint32_t)(p.round - 1), gidx(g, v), p.msg_base + (uint32_t)m,
                     (uint32_t)dv, p.fanout, p.gseed_lo, p.gseed_hi, pk);
        bool hit = false;
        for (int q = 0; q < p.fanout; ++q) hit |= (pk[q] == (uint32_t)lo);
        if (!hit) continue;
      }
    }
    return v;
  }
  return -2;
}

__global__ __launch_bounds__(256) void k_record(DevGraph g, DevState st, RoundParams p) {
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int cur = p.round & 1;
  const int W = st.W;
  const int64_t ntasks = (g.V + 31) >> 5;
  const int nslices = (W + 63) >> 6;
  for (int64_t task = (int64_t)blockIdx.x * WPB + wib; task < ntasks;
       task += (int64_t)gridDim.x * WPB) {
    uint32_t aw = st.A[cur][task];
    while (aw) {
      const int b = __builtin_ctz(aw);
      aw &= aw - 1u;
      const int64_t u = (task << 5) + b;
      for (int sl = 0; sl < nslices; ++sl) {
        const int w = sl * 64 + lane;
        uint64_t f = w < W ? st.F[cur][u * W + w] : 0ull;
        while (f) {
          const int bit = __builtin_ctzll(f);
          f &= f - 1ull;
          const int m = w * 64 + bit;
          st.hop[u * st.M + m] = p.round;
          st.parent[u * st.M + m] = p.round == 0 ? -1 : find_parent(g, st, p, u, m);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_deliveries(DevGraph g, DevState st, RoundParams p,
                                                    int64_t cap, int32_t* peer, int32_t* msg,
                                                    int32_t* parent,
                                                    unsigned long long* counter) {
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int cur = p.round & 1;
  const int W = st.W;
  const int64_t ntasks = (g.V + 31) >> 5;
  const int nslices = (W + 63) >> 6;
  for (int64_t task = (int64_t)blockIdx.x * WPB + wib; task < ntasks;
       task += (int64_t)gridDim.x * WPB) {
    uint32_t aw = st.A[cur][task];
    while (aw) {
      const int b = __builtin_ctz(aw);
      aw &= aw - 1u;
      const int64_t u = (task << 5) + b;
      for (int sl = 0; sl < nslices; ++sl) {
        const int w = sl * 64 + lane;
        uint64_t f = w < W ? st.F[cur][u * W + w] : 0ull;
        while (f) {
          const int bit = __builtin_ctzll(f);
          f &= f - 1ull;
          const int m = w * 64 + bit;
          const unsigned long long pos = atomicAdd(counter, 1ull);
          if ((int64_t)pos < cap) {
            peer[pos] = (int32_t)u;
            msg[pos] = m;
            parent[pos] = p.round == 0 ? -1 : find_parent(g, st, p, u, m);
          }
        }
      }
    }
  }
}

// Vertex-partitioned runs.  plane 0: boundary frontier rows of round `round` out (inactive
// rows as zeros) / ghost frontier rows in (+ A bits).  plane 1 (gossip): pushes pending for
// round `round`+1 into ghost rows out (cleared locally with their T bits) / ORed into the
// owner's rows in (+ T bits).  One wave per row, lane = word.
__global__ __launch_bounds__(256) void k_pack(DevState st, int plane, int round,
                                              const int32_t* __restrict__ ids, int64_t n,
                                              uint64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int W = st.W;
  const int64_t nw = (int64_t)gridDim.x * WPB;
  for (int64_t i = (int64_t)blockIdx.x * WPB + wave_in_block(); i < n; i += nw) {
    const int64_t v = ids[i];
    if (plane == 0) {
      const bool act = bit_test(st.A[round & 1], v);
      for (int w = lane; w < W; w += 64) out[i * W + w] = act ? st.F[round & 1][v * W + w] : 0ull;
    } else {
      uint64_t* nx = st.next[(round + 1) & 1];
      for (int w = lane; w < W; w += 64) {
        out[i * W + w] = nx[v * W + w];
        nx[v * W + w] = 0ull;
      }
      if (lane == 0) atomicAnd(&st.T[(round + 1) & 1][v >> 5], ~(1u << (v & 31)));
    }
  }
}

__global__ __launch_bounds__(256) void k_unpack(DevState st, int plane, int round,
                                                const int32_t* __restrict__ ids, int64_t n,
                                                const uint64_t* __restrict__ in) {
  const int lane = threadIdx.x & 63;
  const int W = st.W;
  const int64_t nw = (int64_t)gridDim.x * WPB;
  for (int64_t i = (int64_t)blockIdx.x * WPB + wave_in_block(); i < n; i += nw) {
    const int64_t v = ids[i];
    bool any = false;
    for (int w = lane; w < W; w += 64) {
      const uint64_t x = in[i * W + w];
      any |= x != 0ull;
      if (plane == 0) st.F[round & 1][v * W + w] = x;
      else if (x) atomicOr((unsigned long long*)&st.next[(round + 1) & 1][v * W + w], (unsigned long long)x);
    }
    if (__ballot(any) && lane == 0) {
      if (plane == 0) atomicOr(&st.A[round & 1][v >> 5], 1u << (v & 31));
      else atomicOr(&st.T[(round + 1) & 1][v >> 5], 1u << (v & 31));
    }
  }
}

// Compacted exchange (vertex-partitioned runs): only live rows travel, as records
// [index in the destination's list segment][W words].  plane 0: frontier rows of round `round`
// (live = A bit) of the send list; plane 1: gossip pushes pending for round+1 in ghost rows
// (live = T bit; row and bit are cleared here).  One wave per 64 list entries (lane = entry)
// computes liveness and destination segment, reserves record slots with one atomic per
// (wave, segment), then copies each live row with lane = word.
__global__ __launch_bounds__(256) void k_pack_live(DevState st, int plane, int round,
                                                   const int32_t* __restrict__ ids, int64_t n,
                                                   const int64_t* __restrict__ seg_off, int nseg,
                                                   unsigned long long* __restrict__ seg_cnt,
                                                   int64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int W = st.W;
  const int64_t R = 1 + W;  // int64 per record
  const int64_t nwaves = (int64_t)gridDim.x * WPB;
  uint64_t* __restrict__ src = plane == 0 ? st.F[round & 1] : st.next[(round + 1) & 1];
  uint32_t* __restrict__ bits = plane == 0 ? st.A[round & 1] : st.T[(round + 1) & 1];
  for (int64_t base = ((int64_t)blockIdx.x * WPB + wave_in_block()) * 64; base < n; base += nwaves * 64) {
    const int64_t i = base + lane;
    const bool valid = i < n;
    const int64_t v = valid ? ids[i] : 0;
    const bool live = valid && bit_test(bits, v);
    int seg = 0;
    for (int q = 1; q < nseg; ++q) seg += i >= ldc(seg_off + q);
    int64_t pos = 0;  // record slot within the segment
    uint64_t todo = __ballot(live);
    while (todo) {
      const int q0 = __builtin_amdgcn_readlane(seg, __builtin_ctzll(todo));
      const uint64_t m = __ballot(live && seg == q0);
      unsigned long long b0 = 0;
      if (lane == 0) b0 = atomicAdd(&seg_cnt[q0], (unsigned long long)__popcll(m));
      b0 = (unsigned long long)readlane64((int64_t)b0, 0);
      if (live && seg == q0)
        pos = (int64_t)b0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      todo &= ~m;
    }
    uint64_t lv = __ballot(live);
    while (lv) {
      const int l = __builtin_ctzll(lv);
      lv &= lv - 1ull;
      const int64_t vl = readlane64(v, l);
      const int sq = __builtin_amdgcn_readlane(seg, l);
      const int64_t rec = (ldc(seg_off + sq) + readlane64(pos, l)) * R;
      if (lane == 0) out[rec] = readlane64(i, l) - ldc(seg_off + sq);
      for (int w = lane; w < W; w += 64) {
        out[rec + 1 + w] = (int64_t)src[vl * W + w];
        if (plane == 1) src[vl * W + w] = 0ull;
      }
      if (plane == 1 && lane == 0) atomicAnd(&bits[vl >> 5], ~(1u << (vl & 31)));
    }
  }
}

// The receiving side: record i came from source rank p with rec_off[p] <= i < rec_off[p+1];
// its index selects the peer in that rank's segment of the list (plane 0: ghosts by owner,
// rows stored + A bit; plane 1: owned boundary peers by neighbour rank, rows ORed + T bit).
struct RecOffsets {
  int64_t off[P2PG_MAX_RANKS + 1];
};

__global__ __launch_bounds__(256) void k_unpack_live(DevState st, int plane, int round,
                                                     const int32_t* __restrict__ ids,
                                                     const int64_t* __restrict__ list_off, int nseg,
                                                     RecOffsets ro, const int64_t* __restrict__ in) {
  const int lane = threadIdx.x & 63;
  const int W = st.W;
  const int64_t R = 1 + W;
  const int64_t nrec = ro.off[nseg];
  for (int64_t i = (int64_t)blockIdx.x * WPB + wave_in_block(); i < nrec; i += (int64_t)gridDim.x * WPB) {
    int p = 0;
    for (int q = 1; q < nseg; ++q) p += i >= ro.off[q];
    const int64_t idx = ldc(in + i * R);
    // a record must name a row of its source's list segment (the host checked the counts; a
    // corrupt index is dropped here rather than written out of bounds)
    if (idx < 0 || idx >= ldc(list_off + p + 1) - ldc(list_off + p)) continue;
    const int64_t v = ids[ldc(list_off + p) + idx];
    for (int w = lane; w < W; w += 64) {
      const uint64_t x = (uint64_t)in[i * R + 1 + w];
      if (plane == 0) st.F[round & 1][v * W + w] = x;
      else if (x) atomicOr((unsigned long long*)&st.next[(round + 1) & 1][v * W + w], (unsigned long long)x);
    }
    if (lane == 0) {
      if (plane == 0) atomicOr(&st.A[round & 1][v >> 5], 1u << (v & 31));
      else atomicOr(&st.T[(round + 1) & 1][v >> 5], 1u << (v & 31));
    }
  }
}

__global__ void k_column(const uint64_t* __restrict__ plane, int32_t W, int32_t w, int64_t V,
                         uint64_t* __restrict__ out) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V;
       v += (int64_t)gridDim.x * blockDim.x)
    out[v] = plane[v * W + w];
}

__global__ void k_philox(int32_t n, const uint32_t* ctr, uint32_t k0, uint32_t k1,
                         uint32_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u32x4 c = {ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]};
  u32x4 r = philox4x32_10(c, k0, k1);
  out[4 * i] = r.x;
  out[4 * i + 1] = r.y;
  out[4 * i + 2] = r.z;
  out[4 * i + 3] = r.w;
}

}  // namespace

hipError_t launch_zero_rows(uint64_t* plane, int32_t W, const int32_t* rows, int32_t n,
                            hipStream_t s) {
  const int64_t tot = (int64_t)n * W;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(k_zero_rows, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, plane,
                     W, rows, n);
  return hipGetLastError();
}

hipError_t launch_seed(const DevState& st, const int32_t* src, int32_t M, hipStream_t s) {
  if (M == 0) return hipSuccess;
  hipLaunchKernelGGL(k_seed, dim3((M + 255) / 256), dim3(256), 0, s, st, src, M);
  return hipGetLastError();
}

template <bool CHURN, bool GOSSIP>
hipError_t pull_with_hubs(const DevGraph& g, const DevState& st, const RoundParams& p,
                          const HubPlan& hp, hipStream_t s) {
  const int grid = grid_tasks((g.V + 31) >> 5);
  if (st.W <= 64) {
    // hubs (deg > HUB_T) are pulled whole in the last phase of a round (phase -1 or 1)
    if (hp.n_items && p.phase != 0)
      launch_hub_partial<CHURN, GOSSIP>(g, st, p, hp, s);
    hipLaunchKernelGGL((k_pull1<CHURN, GOSSIP>),
                       dim3(balanced_grid(k_pull1<CHURN, GOSSIP>, (g.V + 31) >> 5)), dim3(256), 0,
                       s, g, st, p);
    if (hp.n_hubs && p.phase != 0)
      hipLaunchKernelGGL((k_pull_hub_finalize<GOSSIP>), dim3(grid_tasks(hp.n_hubs)), dim3(256),
                         0, s, g, st, p, hp);
  } else {
    DevGraph g2 = g;
    g2.H = nullptr;  // multi-slice rows: no hub split
    hipLaunchKernelGGL((k_pull<CHURN, GOSSIP>), dim3(grid), dim3(256), 0, s, g2, st, p);
  }
  return hipGetLastError();
}

hipError_t launch_flood_pull(const DevGraph& g, const DevState& st, const RoundParams& p,
                             const HubPlan& hp, hipStream_t s) {
  return p.churn_thr ? pull_with_hubs<true, false>(g, st, p, hp, s)
                     : pull_with_hubs<false, false>(g, st, p, hp, s);
}

// k_gossip_fused by churn / fanout (MODE 0, PART) and width (HALF: W <= 32)
template <bool CH, int KK, int MODE, bool PART>
static void fused_launch(bool half, const DevGraph& g, const DevState& st, const RoundParams& p,
                         hipStream_t s) {
  if (half)
    hipLaunchKernelGGL((k_gossip_fused<CH, KK, MODE, true, PART>),
                       dim3(balanced_grid(k_gossip_fused<CH, KK, MODE, true, PART>, (g.V + 31) >> 5)),
                       dim3(256), 0, s, g, st, p);
  else
    hipLaunchKernelGGL((k_gossip_fused<CH, KK, MODE, false, PART>),
                       dim3(balanced_grid(k_gossip_fused<CH, KK, MODE, false, PART>, (g.V + 31) >> 5)),
                       dim3(256), 0, s, g, st, p);
}

// Partitioned ranks (PART, see internal.h): no hub split (H = nullptr: every peer, hubs included,
// goes through the fused pipeline, whose wide-row chunks handle any degree).
static bool part_launch_ok(const DevGraph& g, const DevState& st, int prv) {
  return g.gid != nullptr && g.rev != nullptr && st.W > GROUPED_W_MAX && st.W <= 64 &&
         st.AW[prv] != nullptr && st.E[0] != st.E[1];
}

static hipError_t launch_gossip_fused_part(const DevGraph& g, const DevState& st,
                                           const RoundParams& p, hipStream_t s) {
  if (!part_launch_ok(g, st, (p.round & 1) ^ 1) || p.phase >= 0) return hipErrorInvalidValue;
  DevGraph g2 = g;
  g2.H = nullptr;
  const bool half = st.W <= 32;
  const bool ch = p.churn_thr != 0;
  switch (p.fanout) {
    case 1: ch ? fused_launch<true, 1, 0, true>(half, g2, st, p, s) : fused_launch<false, 1, 0, true>(half, g2, st, p, s); break;
    case 2: ch ? fused_launch<true, 2, 0, true>(half, g2, st, p, s) : fused_launch<false, 2, 0, true>(half, g2, st, p, s); break;
    case 3: ch ? fused_launch<true, 3, 0, true>(half, g2, st, p, s) : fused_launch<false, 3, 0, true>(half, g2, st, p, s); break;
    case 4: ch ? fused_launch<true, 4, 0, true>(half, g2, st, p, s) : fused_launch<false, 4, 0, true>(half, g2, st, p, s); break;
    default: ch ? fused_launch<true, 0, 0, true>(half, g2, st, p, s) : fused_launch<false, 0, 0, true>(half, g2, st, p, s); break;
  }
  return hipGetLastError();
}

// After a PART gather round: the exchanged row pushes it consumed (next[r&1] rows with a T bit,
// saturated peers' included) are cleared, so the plane is all-zero outside pending pushes again.
// One wave per 64 bitmap words (lane = word), then lane = row word per set bit.
__global__ __launch_bounds__(256) void k_clear_arrivals(DevState st, int32_t round, int64_t nwords) {
  const int lane = threadIdx.x & 63;
  const int W = st.W;
  const int cur = round & 1;
  uint32_t* __restrict__ T = st.T[cur];
  uint64_t* __restrict__ nx = st.next[cur];
  for (int64_t base = ((int64_t)blockIdx.x * WPB + wave_in_block()) * 64; base < nwords;
       base += (int64_t)gridDim.x * WPB * 64) {
    const int64_t i = base + lane;
    const uint32_t t = i < nwords ? T[i] : 0u;
    if (t) T[i] = 0u;
    for (uint64_t m = __ballot(t != 0u); m; m &= m - 1ull) {
      const int l = __builtin_ctzll(m);
      uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)t, l);
      const int64_t w0 = (base + l) << 5;
      while (b) {
        const int64_t u = w0 + __builtin_ctz(b);
        b &= b - 1u;
        if (lane < W) nx[u * W + lane] = 0ull;
      }
    }
  }
}

static bool grouped_enabled();
static bool grouped_pull_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("P2PG_GROUPED_PULL");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

hipError_t launch_gossip_pull(const DevGraph& g, const DevState& st, const RoundParams& p,
                              const HubPlan& hp, hipStream_t s) {
  // packed rows (8 < W <= 64): the pull-only mode of the fused kernel (its pipeline crosses task
  // boundaries; W <= 32: two slots per gather load); P2PG_FUSED_PULL=0 keeps the grouped pull-only
  // kernel (W <= 32) / k_pull1 (A/B only)
  static const bool fused_pull = [] {
    const char* e = std::getenv("P2PG_FUSED_PULL");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  if (g.gid && p.phase < 0) {  // partitioned ranks: the PART pull-only pass, hubs inline
    if (!part_launch_ok(g, st, (p.round & 1) ^ 1)) return hipErrorInvalidValue;
    DevGraph g2 = g;
    g2.H = nullptr;
    RoundParams pp = p;
    pp.store_f = 1;
    fused_launch<false, 0, 3, true>(st.W <= 32, g2, st, pp, s);
    return hipGetLastError();
  }
  if (fused_pull && st.W <= 64 && st.AW[(p.round & 1) ^ 1] && p.phase < 0) {
    RoundParams pp = p;
    // the sparse push of this round reads the frontier rows (its listed words only: whole rows,
    // or the nonzero words when nobody else can observe them, store_f == 2)
    pp.store_f = p.store_f == 2 ? 2 : 1;
    // (K = 0: no picks here, and the relay counters take the run's fanout)
    if (hp.n_items)
      launch_hub_partial<false, true>(g, st, pp, hp, s);
    if (st.W <= 32)
      hipLaunchKernelGGL((k_gossip_fused<false, 0, 3, true>),
                         dim3(balanced_grid(k_gossip_fused<false, 0, 3, true>, (g.V + 31) >> 5)),
                         dim3(256), 0, s, g, st, pp);
    else
      hipLaunchKernelGGL((k_gossip_fused<false, 0, 3>),
                         dim3(balanced_grid(k_gossip_fused<false, 0, 3>, (g.V + 31) >> 5)),
                         dim3(256), 0, s, g, st, pp);
    if (hp.n_hubs)
      hipLaunchKernelGGL((k_pull_hub_finalize<true>), dim3(grid_tasks(hp.n_hubs)), dim3(256), 0,
                         s, g, st, pp, hp);
    return hipGetLastError();
  }
  // narrow rows: several peers per wave (the grouped fused kernel without its pushes); the hubs
  // are left to the hub items as in the fused rounds
  if (grouped_enabled() && grouped_pull_enabled() && st.W <= GROUPED_PULL_W_MAX && p.phase < 0) {
    if (hp.n_items)
      launch_hub_partial<false, true>(g, st, p, hp, s);
    hipError_t r = launch_gossip_pull_grouped(g, st, p, s);
    if (r != hipSuccess) return r;
    if (hp.n_hubs)
      hipLaunchKernelGGL((k_pull_hub_finalize<true>), dim3(grid_tasks(hp.n_hubs)), dim3(256), 0,
                         s, g, st, p, hp);
    return hipGetLastError();
  }
  return pull_with_hubs<false, true>(g, st, p, hp, s);
}

hipError_t launch_materialize(const DevGraph& g, const DevState& st, const RoundParams& p,
                              bool flood, hipStream_t s) {
  const int grid = grid_tasks(g.V);
  if (flood)
    hipLaunchKernelGGL(k_materialize<true>, dim3(grid), dim3(256), 0, s, g, st, p);
  else
    hipLaunchKernelGGL(k_materialize<false>, dim3(grid), dim3(256), 0, s, g, st, p);
  return hipGetLastError();
}

// W <= 32 rows: two touched peers per stage of the pipelined update (P2PG_UPDATE_PAIR=0: one)
static bool update_pair_on() {
  static const bool on = [] {
    const char* e = std::getenv("P2PG_UPDATE_PAIR");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

// 32 < W <= 64 rows: two touched peers per stage of the pipelined update (P2PG_UPDATE_DUAL=0: one)
static bool update_dual_on() {
  static const bool on = [] {
    const char* e = std::getenv("P2PG_UPDATE_DUAL");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

hipError_t launch_gossip_update(const DevGraph& g, const DevState& st, const RoundParams& p,
                                hipStream_t s) {
  // blocks cap (P2PG_UPDATE_GRID): c4 A/B, interleaved, update ms per step: 256 / 512 / 1024 /
  // 2048 (GRID_MAX) / 4096 / 8192 blocks -> 40.8 / 25.7 / 18.25 / 18.7 / 20.0 / 22.9
  static const int64_t cap = [] {
    const char* e = std::getenv("P2PG_UPDATE_GRID");
    const int64_t v = e ? std::atoll(e) : 1024;
    return v > 0 ? v : (int64_t)1024;
  }();
  const int grid = (int)std::min<int64_t>(grid_tasks((g.V + 31) >> 5), cap);
  static const bool pipelined = [] {  // P2PG_UPDATE1=0: the unpipelined kernel (A/B only)
    const char* e = std::getenv("P2PG_UPDATE1");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  static const bool narrow = [] {  // P2PG_UPDATE_G=0: one peer per wave at W <= 32 too (A/B)
    const char* e = std::getenv("P2PG_UPDATE_G");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  // several touched peers per wave up to W = 16; at W = 32 (two per wave) the pipelined
  // one-peer kernel is faster (c4 --msgs 2048, profiles/r03/ab_update_g.txt: 20.4 vs 19.65 ms;
  // W = 16: 10.25 vs 13.95 ms, W = 8: 6.75 vs 12.1 ms)
  static const bool gp = [] {  // P2PG_UPDATE_GP=0: the unpipelined grouped update at W <= 16 (A/B)
    const char* e = std::getenv("P2PG_UPDATE_GP");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  if (narrow && gp && st.W > 4 && st.W <= 16) {
    if (st.W <= 8)
      hipLaunchKernelGGL(k_gossip_update_gp<3>, dim3(grid), dim3(256), 0, s, g, st, p);
    else
      hipLaunchKernelGGL(k_gossip_update_gp<4>, dim3(grid), dim3(256), 0, s, g, st, p);
  } else if (narrow && st.W <= 16) {
    int lw = 0;
    while ((1 << lw) < st.W) ++lw;
    switch (lw) {
      case 0: hipLaunchKernelGGL(k_gossip_update_g<0>, dim3(grid), dim3(256), 0, s, g, st, p); break;
      case 1: hipLaunchKernelGGL(k_gossip_update_g<1>, dim3(grid), dim3(256), 0, s, g, st, p); break;
      case 2: hipLaunchKernelGGL(k_gossip_update_g<2>, dim3(grid), dim3(256), 0, s, g, st, p); break;
      case 3: hipLaunchKernelGGL(k_gossip_update_g<3>, dim3(grid), dim3(256), 0, s, g, st, p); break;
      case 4: hipLaunchKernelGGL(k_gossip_update_g<4>, dim3(grid), dim3(256), 0, s, g, st, p); break;
      default: hipLaunchKernelGGL(k_gossip_update_g<5>, dim3(grid), dim3(256), 0, s, g, st, p); break;
    }
  } else if (st.W <= 32 && pipelined && update_pair_on()) {
    hipLaunchKernelGGL(k_gossip_update1<2>, dim3(grid), dim3(256), 0, s, g, st, p);
  } else if (st.W <= 64 && pipelined && update_dual_on()) {
    hipLaunchKernelGGL(k_gossip_update1<3>, dim3(grid), dim3(256), 0, s, g, st, p);
  } else if (st.W <= 64 && pipelined)
    hipLaunchKernelGGL(k_gossip_update1<1>, dim3(grid), dim3(256), 0, s, g, st, p);
  else
    hipLaunchKernelGGL(k_gossip_update, dim3(grid), dim3(256), 0, s, g, st, p);
  return hipGetLastError();
}

template <bool SE>
void scatter_dispatch(int grid, const DevGraph& g, const DevState& st, const RoundParams& p,
                      const int64_t* hub_items, int64_t n_hub_items, int64_t task0,
                      hipStream_t s) {
  // (partitioned ranks' E stores: ghost connections go to row pushes, scatter_row PART)
  const bool part = SE && g.gid != nullptr;
#define P2PG_SCATTER(CH, KK)                                                                   \
  do {                                                                                         \
    if (part)                                                                                  \
      hipLaunchKernelGGL((k_gossip_scatter<CH, KK, SE, true>), dim3(grid), dim3(256), 0, s, g, \
                         st, p, hub_items, n_hub_items, task0);                                \
    else                                                                                       \
      hipLaunchKernelGGL((k_gossip_scatter<CH, KK, SE>), dim3(grid), dim3(256), 0, s, g, st,   \
                         p, hub_items, n_hub_items, task0);                                    \
  } while (0)
  const bool ch = p.churn_thr != 0;
  switch (p.fanout) {
    case 1: if (ch) P2PG_SCATTER(true, 1); else P2PG_SCATTER(false, 1); break;
    case 2: if (ch) P2PG_SCATTER(true, 2); else P2PG_SCATTER(false, 2); break;
    case 3: if (ch) P2PG_SCATTER(true, 3); else P2PG_SCATTER(false, 3); break;
    case 4: if (ch) P2PG_SCATTER(true, 4); else P2PG_SCATTER(false, 4); break;
    default: if (ch) P2PG_SCATTER(true, 0); else P2PG_SCATTER(false, 0); break;
  }
#undef P2PG_SCATTER
}

static bool grouped_enabled();

// The push modes of the fused / grouped kernels (push-only, update+push) skip the pull hubs
// (g.H: deg > HUB_T) and leave their pushes to launch_wide_push_e over wide_big (the same deg >
// HUB_T set, checked equal when the graph is uploaded).  Both launchers take that path only when
// the hub pushes can actually run: their chunk items and ids are there, and so is the H bitmap.
static bool hub_pushes_ready(const DevGraph& g, const int64_t* big_items, int64_t n_big,
                             const int32_t* wide_big, int64_t n_wide_big) {
  return (n_big == 0 || (big_items && wide_big)) && (n_wide_big == 0 || g.H != nullptr);
}

hipError_t launch_gossip_scatter(const DevGraph& g, const DevState& st, const RoundParams& p,
                                 const int64_t* hub_items, int64_t n_hub_items, bool store_e,
                                 hipStream_t s, const int64_t* big_items, int64_t n_big,
                                 const int32_t* wide_big, int64_t n_wide_big) {
  // blocks cap: P2PG_SCATTER_GRID (default GRID_MAX)
  static const int64_t cap = [] {
    const char* e = std::getenv("P2PG_SCATTER_GRID");
    const int64_t v = e ? std::atoll(e) : GRID_MAX;
    return v > 0 ? v : (int64_t)GRID_MAX;
  }();
  const int grid = (int)std::min<int64_t>(
      grid_tasks_uncapped(((g.V + 31) >> 5) + ((n_hub_items + 63) >> 6)), cap);
  static const bool push_grouped = [] {  // P2PG_PUSH_GROUPED=0: one wave per source (A/B)
    const char* e = std::getenv("P2PG_PUSH_GROUPED");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  const bool hubs_ok = hub_pushes_ready(g, big_items, n_big, wide_big, n_wide_big);
  if (store_e && push_grouped && grouped_enabled() && st.W <= GROUPED_W_MAX && hubs_ok && !g.gid) {
    hipError_t r = launch_gossip_push_grouped(g, st, p, s);
    if (r != hipSuccess) return r;
    return launch_wide_push_e(g, st, p, big_items, n_big, wide_big, n_wide_big, s);
  }
  // wider packed rows: the push-only mode of the one-peer-per-wave fused kernel, hubs by atomics
  // P2PG_PUSH_FUSED=0: one wave per source (A/B; read per launch -- one per run -- so a test can
  // switch it between engines of one process)
  const char* pf_env = std::getenv("P2PG_PUSH_FUSED");
  const bool push_fused = !(pf_env && std::strcmp(pf_env, "0") == 0);
  if (store_e && push_fused && st.W <= 64 && st.AW[p.round & 1] != nullptr && hubs_ok && !g.gid) {
#define P2PG_FUSED_PO(CH, KK)                                                                       \
  hipLaunchKernelGGL((k_gossip_fused<CH, KK, 1>),                                                 \
                     dim3(balanced_grid(k_gossip_fused<CH, KK, 1>, (g.V + 31) >> 5)), dim3(256),    \
                     0, s, g, st, p)
    const bool ch = p.churn_thr != 0;
    switch (p.fanout) {
      case 1: if (ch) P2PG_FUSED_PO(true, 1); else P2PG_FUSED_PO(false, 1); break;
      case 2: if (ch) P2PG_FUSED_PO(true, 2); else P2PG_FUSED_PO(false, 2); break;
      case 3: if (ch) P2PG_FUSED_PO(true, 3); else P2PG_FUSED_PO(false, 3); break;
      case 4: if (ch) P2PG_FUSED_PO(true, 4); else P2PG_FUSED_PO(false, 4); break;
      default: if (ch) P2PG_FUSED_PO(true, 0); else P2PG_FUSED_PO(false, 0); break;
    }
#undef P2PG_FUSED_PO
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) return r;
    return launch_wide_push_e(g, st, p, big_items, n_big, wide_big, n_wide_big, s);
  }
  if (store_e)
    scatter_dispatch<true>(grid, g, st, p, hub_items, n_hub_items, 0, s);
  else
    scatter_dispatch<false>(grid, g, st, p, hub_items, n_hub_items, 0, s);
  return hipGetLastError();
}

// narrow rows (W <= GROUPED_W_MAX: one rank's share of a message split): several peers per
// wave.
// P2PG_GROUPED=0 keeps one wave per peer (A/B only; needs packed rows).
static bool grouped_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("P2PG_GROUPED");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

bool gossip_update_push_supported(const DevState& st) {
  return st.W > 16 && st.W <= 64 && st.AW[0] != nullptr && st.E[0] != nullptr &&
         !(grouped_enabled() && st.W <= GROUPED_W_MAX);
}

hipError_t launch_gossip_update_push(const DevGraph& g, const DevState& st, const RoundParams& p,
                                     const int64_t* big_items, int64_t n_big,
                                     const int32_t* wide_big, int64_t n_wide_big, hipStream_t s) {
  if (!gossip_update_push_supported(st) || p.phase >= 0 ||
      !hub_pushes_ready(g, big_items, n_big, wide_big, n_wide_big))
    return hipErrorInvalidValue;
#define P2PG_FUSED_UP(CH, KK)                                                                       \
  hipLaunchKernelGGL((k_gossip_fused<CH, KK, 2>),                                                 \
                     dim3(balanced_grid(k_gossip_fused<CH, KK, 2>, (g.V + 31) >> 5)), dim3(256),    \
                     0, s, g, st, p)
  const bool ch = p.churn_thr != 0;
  switch (p.fanout) {
    case 1: if (ch) P2PG_FUSED_UP(true, 1); else P2PG_FUSED_UP(false, 1); break;
    case 2: if (ch) P2PG_FUSED_UP(true, 2); else P2PG_FUSED_UP(false, 2); break;
    case 3: if (ch) P2PG_FUSED_UP(true, 3); else P2PG_FUSED_UP(false, 3); break;
    case 4: if (ch) P2PG_FUSED_UP(true, 4); else P2PG_FUSED_UP(false, 4); break;
    default: if (ch) P2PG_FUSED_UP(true, 0); else P2PG_FUSED_UP(false, 0); break;
  }
#undef P2PG_FUSED_UP
  hipError_t r = hipGetLastError();
  if (r != hipSuccess) return r;
  if (g.H) {
    // the touched hubs (left in T): the update's second phase over the hub bitmap, which ORs
    // their activity bits into the words the fused pass wrote
    RoundParams ph = p;
    ph.border = g.H;
    ph.phase = 1;
    const int grid = (int)std::min<int64_t>(grid_tasks((g.V + 31) >> 5), 1024);
    hipLaunchKernelGGL(k_gossip_update1<1>, dim3(grid), dim3(256), 0, s, g, st, ph);
    r = hipGetLastError();
    if (r != hipSuccess) return r;
  }
  return launch_wide_push_e(g, st, p, big_items, n_big, wide_big, n_wide_big, s);
}

bool gossip_fused_supported(const DevState& st) {
  if (st.W > 64 || st.E[0] == st.E[1]) return false;
  return (grouped_enabled() && st.W <= GROUPED_W_MAX) || st.AW[0] != nullptr;
}

hipError_t launch_gossip_fused(const DevGraph& g, const DevState& st, const RoundParams& p,
                               const HubPlan& hp, const int64_t* big_items, int64_t n_big,
                               bool skip_big, hipStream_t s) {
  if (!gossip_fused_supported(st)) return hipErrorInvalidValue;
  if (g.gid) return launch_gossip_fused_part(g, st, p, s);  // (the caller clears the arrivals)
  if (hp.n_items)
    launch_hub_partial<false, true>(g, st, p, hp, s);
  if (grouped_enabled() && st.W <= GROUPED_W_MAX) {
    hipError_t r = launch_gossip_fused_grouped(g, st, p, s);
    if (r != hipSuccess) return r;
  } else {
#define P2PG_FUSED(CH, KK)                                                                       \
  do {                                                                                         \
    if (half)                                                                                  \
      hipLaunchKernelGGL((k_gossip_fused<CH, KK, 0, true>),                                    \
                         dim3(balanced_grid(k_gossip_fused<CH, KK, 0, true>, (g.V + 31) >> 5)), \
                         dim3(256), 0, s, g, st, p);                                           \
    else                                                                                       \
      hipLaunchKernelGGL((k_gossip_fused<CH, KK>),                                             \
                         dim3(balanced_grid(k_gossip_fused<CH, KK>, (g.V + 31) >> 5)), dim3(256), \
                         0, s, g, st, p);                                                      \
  } while (0)
  // W <= 32: two slots per gather load (P2PG_FUSED_HALF=0: one, A/B only)
  static const bool half_on = [] {
    const char* e = std::getenv("P2PG_FUSED_HALF");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  const bool half = half_on && st.W <= 32;
  const bool ch = p.churn_thr != 0;
  switch (p.fanout) {
    case 1: if (ch) P2PG_FUSED(true, 1); else P2PG_FUSED(false, 1); break;
    case 2: if (ch) P2PG_FUSED(true, 2); else P2PG_FUSED(false, 2); break;
    case 3: if (ch) P2PG_FUSED(true, 3); else P2PG_FUSED(false, 3); break;
    case 4: if (ch) P2PG_FUSED(true, 4); else P2PG_FUSED(false, 4); break;
    default: if (ch) P2PG_FUSED(true, 0); else P2PG_FUSED(false, 0); break;
  }
#undef P2PG_FUSED
  }
  if (hp.n_hubs)
    hipLaunchKernelGGL((k_pull_hub_finalize<true>), dim3(grid_tasks(hp.n_hubs)), dim3(256), 0,
                       s, g, st, p, hp);
  if (n_big && !skip_big) {
    const int64_t nwords = (g.V + 31) >> 5;
    scatter_dispatch<true>(grid_tasks((n_big + 63) >> 6), g, st, p, big_items, n_big, nwords, s);
  }
  return hipGetLastError();
}

hipError_t launch_clear_arrivals(const DevState& st, int32_t round, int64_t V, hipStream_t s) {
  const int64_t nwords = (V + 31) >> 5;
  hipLaunchKernelGGL(k_clear_arrivals, dim3(grid_tasks((nwords + 63) >> 6)), dim3(256), 0, s, st,
                     round, nwords);
  return hipGetLastError();
}

hipError_t launch_record(const DevGraph& g, const DevState& st, const RoundParams& p,
                         hipStream_t s) {
  const int grid = grid_tasks((g.V + 31) >> 5);
  hipLaunchKernelGGL(k_record, dim3(grid), dim3(256), 0, s, g, st, p);
  return hipGetLastError();
}

hipError_t launch_deliveries(const DevGraph& g, const DevState& st, const RoundParams& p,
                             int64_t cap, int32_t* peer, int32_t* msg, int32_t* parent,
                             unsigned long long* counter, hipStream_t s) {
  const int grid = grid_tasks((g.V + 31) >> 5);
  hipLaunchKernelGGL(k_deliveries, dim3(grid), dim3(256), 0, s, g, st, p, cap, peer, msg,
                     parent, counter);
  return hipGetLastError();
}

hipError_t launch_pack(const DevState& st, int plane, int round, const int32_t* ids, int64_t n,
                       uint64_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack, dim3(grid_tasks(n)), dim3(256), 0, s, st, plane, round, ids, n, out);
  return hipGetLastError();
}

hipError_t launch_unpack(const DevState& st, int plane, int round, const int32_t* ids, int64_t n,
                         const uint64_t* in, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack, dim3(grid_tasks(n)), dim3(256), 0, s, st, plane, round, ids, n, in);
  return hipGetLastError();
}

hipError_t launch_pack_live(const DevState& st, int plane, int round, const int32_t* ids, int64_t n,
                            const int64_t* seg_off, int nseg, unsigned long long* seg_cnt,
                            int64_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t waves = (n + 63) / 64;
  hipLaunchKernelGGL(k_pack_live, dim3(grid_tasks(waves)), dim3(256), 0, s, st, plane, round, ids, n,
                     seg_off, nseg, seg_cnt, out);
  return hipGetLastError();
}

hipError_t launch_unpack_live(const DevState& st, int plane, int round, const int32_t* ids,
                              const int64_t* list_off, int nseg, const int64_t* rec_off,
                              const int64_t* in, hipStream_t s) {
  if (nseg < 1 || nseg > P2PG_MAX_RANKS) return hipErrorInvalidValue;
  RecOffsets ro{};
  for (int q = 0; q <= nseg; ++q) ro.off[q] = rec_off[q];
  if (ro.off[nseg] <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack_live, dim3(grid_tasks(ro.off[nseg])), dim3(256), 0, s, st, plane, round,
                     ids, list_off, nseg, ro, in);
  return hipGetLastError();
}

hipError_t launch_column(const uint64_t* plane, int32_t W, int32_t w, int64_t V, uint64_t* out,
                         hipStream_t s) {
  if (V <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((V + 255) / 256, 8192);
  hipLaunchKernelGGL(k_column, dim3((unsigned)blocks), dim3(256), 0, s, plane, W, w, V, out);
  return hipGetLastError();
}

hipError_t launch_philox(int32_t n, const uint32_t* ctr, uint32_t k0, uint32_t k1,
                         uint32_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_philox, dim3((n + 255) / 256), dim3(256), 0, s, n, ctr, k0, k1, out);
  return hipGetLastError();
}

}  // namespace p2pg
