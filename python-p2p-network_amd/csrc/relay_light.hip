// Light dense gossip rounds, one LANE per peer (k_gossip_light).
//
// Why: the fused dense round (k_gossip_fused, relay_kernels.hip) gives every visited peer a whole
// wave -- lane = word of its 64-word row -- and spends ~355 VALU instructions of fixed per-peer
// work on it (slot readlanes, gather setup, ballots, compaction, a 64-lane pick batch, table
// clear, flush).  In the light rounds of config 4 (the first fused rounds after the sparse phase
// and the last ones before it) a peer carries 8-30 arrival words and 8-50 new bits, so most of
// those lanes idle and the round is VALU-bound at a fraction of the HBM rate.
// Here the low-degree peers of such a round (deg <= LIGHT_DEG: ~94 % of a Barabasi-Albert m=4
// graph) are taken 64 to a wave, lane = peer, each lane walking its own peer's work serially:
//   1. its <= LIGHT_DEG connections: neighbour ids, activity bits and active-word masks (AW of
//      round r-1), all loads of a step issued back to back; the masks go to a per-lane LDS column;
//   2. per arrival word w (the union of the masks): its seen word and the packed E words of the
//      active connections holding w (issued together), dedup -> first receipts, seen / frontier
//      words, counters;
//   3. per new word (rank i of the peer's new active-word mask): the Philox picks of its bits
//       ORed into the lane's LDS column of per-connection masks, then one packed
//      E store per connection at rank i (receiver-major slot rev[j], zeros included, churn-dropped
//      connections zero) -- exactly the rows k_gossip_fused would write.
// The rest of the round (higher-degree peers, hubs) runs through k_gossip_fused as usual, which
// skips the light peers (RoundParams::light); this kernel runs after it and ORs its activity bits
// into the task words.  Same outputs and counters; saturation bits are left unset for the light
// peers (a hint that lets later rounds skip a peer, never a result).  Reference semantics: the
// relay of first receipts by Node.send_to_node on the chosen connections (node.py:114-120), lost
// sends over dropped connections (nodeconnection.py:123-126).
#include "device_util.h"

namespace p2pg {
namespace {

template <bool CHURN, int K>
__global__ __launch_bounds__(256) void k_gossip_light(DevGraph g, DevState st, RoundParams p) {
  constexpr int D = LIGHT_DEG;
  // per wave, [connection][lane]: round r-1 active-word masks (step 1-2), then pick masks (3);
  // lane-minor so the 64 lanes of an access hit 64 consecutive 8-byte words
  __shared__ uint64_t tab_all[WPB][D][64];
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  uint64_t(*tab)[64] = tab_all[wib];
  const int64_t V = g.V;
  const int W = st.W;
  const int cur = p.round & 1, prv = cur ^ 1;
  const uint64_t* __restrict__ Src = st.E[prv];
  uint64_t* __restrict__ Eo = st.E[cur];
  uint64_t* __restrict__ Fc = st.F[cur];
  const uint32_t* __restrict__ Ap = st.A[prv];
  const uint64_t* __restrict__ AWp = st.AW[prv];
  const uint32_t kf = K > 0 ? (uint32_t)K : (uint32_t)p.fanout;
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t ngroups = (V + 63) >> 6;
  for (int64_t grp = (int64_t)blockIdx.x * WPB + wib; grp < ngroups; grp += (int64_t)gridDim.x * WPB) {
    const int64_t u = (grp << 6) + lane;
    bool ok = false;
    if (u < V) {
      const int64_t t = u >> 5;
      ok = ((p.light[t] & ~st.S[t]) >> (u & 31)) & 1u;
    }
    if (!__ballot(ok)) continue;
    int64_t beg = 0;
    int deg = 0;
    if (ok) {
      beg = g.rowptr[u];
      deg = (int)(g.rowptr[u + 1] - beg);
    }
    // 1. connections
    int32_t nb[D];
#pragma unroll
    for (int j = 0; j < D; ++j) nb[j] = j < deg ? g.colidx[beg + j] : 0;
    uint32_t aw[D];
#pragma unroll
    for (int j = 0; j < D; ++j) aw[j] = j < deg ? Ap[nb[j] >> 5] : 0u;
    uint64_t uni = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const bool act = (aw[j] >> (nb[j] & 31)) & 1u;
      const uint64_t am = act ? AWp[nb[j]] : 0ull;
      tab[j][lane] = am;
      uni |= am;
    }
    // 2. arrivals, dedup, first receipts
    uint64_t* const seenu = st.seen + u * W;
    uint64_t* const Fu = Fc + u * W;
    const uint32_t per_bit = (uint32_t)deg < kf ? (uint32_t)deg : kf;
    uint64_t wm = 0;
    uint64_t rem = uni;
    while (__ballot(rem != 0ull)) {
      const bool has = rem != 0ull;
      const int w = has ? __builtin_ctzll(rem) : 0;
      rem &= rem - 1ull;
      const uint64_t below = (1ull << w) - 1ull;
      const uint64_t s = has ? seenu[w] : ~0ull;
      uint64_t acc = 0;
#pragma unroll
      for (int j = 0; j < D; ++j) {
        const uint64_t am = tab[j][lane];
        if (has && ((am >> w) & 1ull)) acc |= Src[(beg + j) * W + __popcll(am & below)];
      }
      const uint64_t nw = acc & full_mask(w, W, st.M) & ~s;
      if (nw) {
        st_frow(&seenu[w], s | nw);
        Fu[w] = nw;  // (read back below)
        const uint32_t pc = (uint32_t)__popcll(nw);
        c[ST_NEW] += pc;
        c[ST_RELAYS] += (uint64_t)pc * per_bit;
        c[ST_ACTIVE_W] += 1;
        c[ST_WEDGES] += (uint64_t)deg;
        wm |= 1ull << w;
      }
    }
    const uint64_t actm = __ballot(wm != 0ull);
    if (!actm) continue;
    if (wm) {
      st.AW[cur][u] = wm;
      c[ST_ACTIVE_V] += 1;
      c[ST_DEG_ACT] += (uint64_t)deg;
    }
    if (lane == 0 && (uint32_t)actm) atomicOr(&st.A[cur][grp << 1], (uint32_t)actm);
    if (lane == 32 && (uint32_t)(actm >> 32)) atomicOr(&st.A[cur][(grp << 1) + 1], (uint32_t)(actm >> 32));
    // 3. pushes of the new words, rank by rank
    uint32_t rv[D];
#pragma unroll
    for (int j = 0; j < D; ++j) rv[j] = (wm && j < deg) ? g.rev[beg + j] : 0u;
    uint32_t drop = 0;
    if (CHURN && wm) {
#pragma unroll
      for (int j = 0; j < D; ++j)
        if (j < deg && churn_dropped((uint32_t)p.round, (uint32_t)u, (uint32_t)nb[j], p.churn_thr,
                                     p.cseed_lo, p.cseed_hi))
          drop |= 1u << j;
    }
    const bool all = (uint32_t)deg <= kf;
    uint64_t remw = wm;
    int rank = 0;
    while (__ballot(remw != 0ull)) {
      const bool has = remw != 0ull;
      const int w = has ? __builtin_ctzll(remw) : 0;
      remw &= remw - 1ull;
      const uint64_t nw = has ? Fu[w] : 0ull;
      if (!all) {
#pragma unroll
        for (int j = 0; j < D; ++j) tab[j][lane] = 0ull;
        uint64_t bits = nw;
        while (__ballot(bits != 0ull)) {
          if (bits) {
            const int b = __builtin_ctzll(bits);
            bits &= bits - 1ull;
            const uint32_t mg = p.msg_base + (uint32_t)(w * 64 + b);
            if constexpr (K > 0) {
              uint32_t pk[K];
              gossip_picks_t<K>((uint32_t)p.round, (uint32_t)u, mg, (uint32_t)deg, p.gseed_lo, p.gseed_hi, pk);
#pragma unroll
              for (int q = 0; q < K; ++q) tab[pk[q]][lane] |= 1ull << b;
            } else {
              uint32_t pk[16];
              gossip_picks((uint32_t)p.round, (uint32_t)u, mg, (uint32_t)deg, (int)kf, p.gseed_lo, p.gseed_hi, pk);
              for (uint32_t q = 0; q < kf; ++q) tab[pk[q]][lane] |= 1ull << b;
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < D; ++j) {
        if (has && j < deg) {
          const bool dropped = CHURN && ((drop >> j) & 1u);
          const uint64_t x = dropped ? 0ull : (all ? nw : tab[j][lane]);
          st_row(&Eo[(int64_t)rv[j] * W + rank], x);
          c[ST_SCATTER] += x != 0ull;
        }
      }
      rank += has ? 1 : 0;
    }
    // whole frontier rows where they are observed (RoundParams::store_f == 1): zero the words
    // with no first receipt, one row per instruction
    if (p.store_f == 1) {
      uint64_t pm = actm;
      while (pm) {
        const int l = __builtin_ctzll(pm);
        pm &= pm - 1ull;
        const uint64_t wml = (uint64_t)readlane64((int64_t)wm, l);
        if (lane < W && !((wml >> lane) & 1ull)) Fc[((grp << 6) + l) * W + lane] = 0ull;
      }
    }
  }
  flush_stats(st.stats, c, lane);
}

}  // namespace

bool gossip_light_supported(const DevState& st) {
  return st.W > GROUPED_W_MAX && st.W <= 64 && st.AW[0] != nullptr && st.E[0] != nullptr &&
         st.E[0] != st.E[1];
}

hipError_t launch_gossip_light(const DevGraph& g, const DevState& st, const RoundParams& p, hipStream_t s) {
  if (!p.light || !gossip_light_supported(st) || g.gid) return hipErrorInvalidValue;
  const int64_t ngroups = (g.V + 63) >> 6;
  const int blocks = (int)std::min<int64_t>((ngroups + WPB - 1) / WPB, 8192);
  const bool ch = p.churn_thr != 0;
#define P2PG_LIGHT(CH, KK) \
  hipLaunchKernelGGL((k_gossip_light<CH, KK>), dim3(blocks), dim3(256), 0, s, g, st, p)
  switch (p.fanout) {
    case 1: if (ch) P2PG_LIGHT(true, 1); else P2PG_LIGHT(false, 1); break;
    case 2: if (ch) P2PG_LIGHT(true, 2); else P2PG_LIGHT(false, 2); break;
    case 3: if (ch) P2PG_LIGHT(true, 3); else P2PG_LIGHT(false, 3); break;
    case 4: if (ch) P2PG_LIGHT(true, 4); else P2PG_LIGHT(false, 4); break;
    default: if (ch) P2PG_LIGHT(true, 0); else P2PG_LIGHT(false, 0); break;
  }
#undef P2PG_LIGHT
  return hipGetLastError();
}

}  // namespace p2pg
