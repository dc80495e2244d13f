// The sends of one round, as the reference makes them: every Node.send_to_node call
// (p2pnetwork/node.py:114-120) that the round's first receipts cause, and which of them never
// arrive.  Used by
//   * the arrival counter p2pg_round_stats.received (NodeConnection.run's message_count_recv,
//     nodeconnection.py:215): sends of the round before minus those lost to churn (the send
//     over a broken link, nodeconnection.py:123-126) or to a removed connection;
//   * the per-callback compat mode: p2pg_get_sends hands every (sender, receiver, msg) of a
//     round to the host, which calls node_message once per arrival (nodeconnection.py:211-216),
//     and p2pg_drop_relays withdraws the relays of first receipts whose app did not forward.
// Validation-scale paths (compat graphs) and a counting pass for churn runs; the rounds' own
// kernels never depend on them.  Internal; not part of the C-ABI.
#include "device_util.h"

namespace p2pg {
namespace {

// Did neighbour y's round-(r-1) send of this lane's word reach v?  (find_parent's test, word-wide:
// y relayed in round r-1 -- its A bit and frontier word --, the connection was not removed
// before the messages arrived, and churn did not drop it.)  Flood only; wave-uniform y.
__device__ __forceinline__ uint64_t prev_sends(const DevGraph& gp, const DevState& st, const RoundParams& p,
                                               int64_t v, int32_t y, int64_t slot, int w) {
  const int prv = (p.round & 1) ^ 1;
  if (gp.gone && gp.gone[slot]) return 0ull;
  if (!bit_test(st.A[prv], y)) return 0ull;
  if (p.churn_thr && churn_dropped((uint32_t)(p.round - 1), gidx(gp, v), gidx(gp, y), p.churn_thr,
                                   p.cseed_lo, p.cseed_hi))
    return 0ull;
  return w < st.W ? st.F[prv][(int64_t)y * st.W + w] : 0ull;
}

__device__ __forceinline__ bool send_lost(const DevGraph& gs, const RoundParams& p, int64_t v, int32_t u,
                                          int64_t slot) {
  if (gs.gone && gs.gone[slot]) return true;
  return p.churn_thr && churn_dropped((uint32_t)p.round, gidx(gs, v), gidx(gs, u), p.churn_thr,
                                      p.cseed_lo, p.cseed_hi);
}

// One wave per active peer v of round r = p.round (A[r&1]), lane = word of a 64-word slice.
// Flood: v sends every first receipt m to each connection over gs but the sender it first got m
// from -- the lowest-id neighbour over gp whose round-(r-1) send reached it (exclude=[sender],
// node.py:106-112; none at the origin, r = 0).  Walking v's gp row ascending, `rem` holds the
// bits whose sender is not found yet; a neighbour y takes rem & (y's sends) as its own.
// Gossip: one send per Philox pick (the sender is not excluded).
// EMIT: records at atomic positions (< cap); else only the lost sends are counted (cnt[1]) and
// peers without a lost connection are skipped.  cnt[0] = sends emitted.
template <bool EMIT>
__global__ __launch_bounds__(256) void k_sends(DevGraph gs, DevGraph gp, DevState st, RoundParams p,
                                               int64_t cap, int32_t* __restrict__ snd,
                                               int32_t* __restrict__ rcv, int32_t* __restrict__ msg,
                                               uint8_t* __restrict__ lostf,
                                               unsigned long long* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  const int cur = p.round & 1;
  const int W = st.W;
  const int nslices = (W + 63) >> 6;
  const int64_t ntasks = (gs.V + 31) >> 5;
  unsigned long long n_lost = 0, n_sent = 0;
  auto put = [&](int64_t v, int32_t u, int m, bool l) {
    if (EMIT) {
      const unsigned long long pos = atomicAdd(cnt, 1ull);
      if ((int64_t)pos < cap) {
        snd[pos] = (int32_t)v;
        rcv[pos] = u;
        msg[pos] = m;
        lostf[pos] = l ? 1 : 0;
      }
    }
  };
  for (int64_t task = (int64_t)blockIdx.x * WPB + wib; task < ntasks; task += (int64_t)gridDim.x * WPB) {
    uint32_t aw = st.A[cur][task];
    while (aw) {
      const int b = __builtin_ctz(aw);
      aw &= aw - 1u;
      const int64_t v = (task << 5) + b;
      const int64_t beg = gs.rowptr[v], end = gs.rowptr[v + 1];
      if (beg == end) continue;
      int64_t last_lost = end;  // count mode: the walk stops after the last lost connection
      if (!EMIT) {
        last_lost = -1;
        for (int64_t j0 = beg; j0 < end; j0 += 64) {
          const int64_t j = j0 + lane;
          const bool l = j < end && send_lost(gs, p, v, gs.colidx[j], j);
          const uint64_t bl = __ballot(l);
          if (bl) last_lost = j0 + 63 - __builtin_clzll(bl);
        }
        if (last_lost < 0) continue;
        last_lost += 1;
      }
      for (int sl = 0; sl < nslices; ++sl) {
        const int w = sl * 64 + lane;
        const uint64_t f = w < W ? st.F[cur][v * W + w] : 0ull;
        if (!__ballot(f != 0ull)) continue;
        if (p.mode == 0) {
          uint64_t rem = p.round > 0 ? f : 0ull;
          int64_t jp = gp.rowptr[v];
          const int64_t ep = gp.rowptr[v + 1];
          for (int64_t j = beg; j < last_lost; ++j) {
            const int32_t u = gs.colidx[j];
            uint64_t pu = 0ull;  // bits whose sender is u: not sent back to it
            while (jp < ep) {
              const int32_t y = gp.colidx[jp];
              if (y > u) break;
              const uint64_t sy = __ballot(rem != 0ull) ? prev_sends(gp, st, p, v, y, jp, w) : 0ull;
              if (y == u) pu = rem & sy;
              rem &= ~sy;
              ++jp;
              if (y == u) break;
            }
            const uint64_t out = f & ~pu;
            const bool l = send_lost(gs, p, v, u, j);
            if (EMIT) {
              uint64_t o = out;
              while (o) {
                const int bit = __builtin_ctzll(o);
                o &= o - 1ull;
                put(v, u, w * 64 + bit, l);
              }
            } else if (l) {
              n_lost += (unsigned long long)__popcll(out);
            }
          }
        } else {
          const uint32_t deg = (uint32_t)(end - beg);
          uint64_t o = f;
          while (o) {
            const int bit = __builtin_ctzll(o);
            o &= o - 1ull;
            const int m = w * 64 + bit;
            uint32_t pk[16];
            const int k = (int)deg <= p.fanout ? (int)deg : p.fanout;
            if ((int)deg > p.fanout)
              gossip_picks((uint32_t)p.round, gidx(gs, v), p.msg_base + (uint32_t)m, deg, p.fanout,
                           p.gseed_lo, p.gseed_hi, pk);
            for (int q = 0; q < k; ++q) {
              const int64_t j = beg + ((int)deg > p.fanout ? (int64_t)pk[q] : (int64_t)q);
              const int32_t u = gs.colidx[j];
              const bool l = send_lost(gs, p, v, u, j);
              put(v, u, m, l);
              n_lost += l ? 1u : 0u;
              n_sent += 1u;
            }
          }
        }
      }
    }
  }
  if (!EMIT) {
    const unsigned long long tl = wave_sum(n_lost);
    if (lane == 0 && tl) atomicAdd(cnt + 1, tl);
  }
  (void)n_sent;
}

// p2pg_drop_relays: how many listed (peer, msg) bits are set in the last round's frontier
// (check), then clear them (check = false).  list[i] = (peer << 32) | msg.
__global__ __launch_bounds__(256) void k_drop(DevState st, int32_t round, const uint64_t* __restrict__ list,
                                              int64_t n, bool check, unsigned long long* __restrict__ hits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int cur = round & 1;
  unsigned long long h = 0;
  if (i < n) {
    const int64_t v = (int64_t)(list[i] >> 32);
    const int m = (int)(uint32_t)list[i];
    const uint64_t bit = 1ull << (m & 63);
    uint64_t* word = &st.F[cur][v * st.W + (m >> 6)];
    if (check)
      h = (bit_test(st.A[cur], v) && (*word & bit)) ? 1u : 0u;
    else
      atomicAnd((unsigned long long*)word, ~(unsigned long long)bit);
  }
  if (check) {
    const unsigned long long t = wave_sum(h);
    if ((threadIdx.x & 63) == 0 && t) atomicAdd(hits, t);
  }
}

// AW[cur][v] = the nonzero words of F[cur][v] (W <= 64) for the active rows of round `round`
// (after a drop, and after a restore: snapshots carry F, not its word masks).
__global__ __launch_bounds__(256) void k_rebuild_aw(DevState st, int32_t round, int64_t V) {
  const int lane = threadIdx.x & 63;
  const int cur = round & 1;
  const int64_t ntasks = (V + 31) >> 5;
  for (int64_t task = (int64_t)blockIdx.x * WPB + wave_in_block(); task < ntasks;
       task += (int64_t)gridDim.x * WPB) {
    uint32_t aw = st.A[cur][task];
    while (aw) {
      const int b = __builtin_ctz(aw);
      aw &= aw - 1u;
      const int64_t v = (task << 5) + b;
      const uint64_t f = lane < st.W ? st.F[cur][v * st.W + lane] : 0ull;
      const uint64_t m = __ballot(f != 0ull);
      if (lane == 0) st.AW[cur][v] = m;
    }
  }
}

}  // namespace

hipError_t launch_sends(const DevGraph& gs, const DevGraph& gp, const DevState& st, const RoundParams& p,
                        bool emit, int64_t cap, int32_t* snd, int32_t* rcv, int32_t* msg, uint8_t* lost,
                        unsigned long long* cnt, hipStream_t s) {
  const int grid = grid_tasks((gs.V + 31) >> 5);
  if (emit)
    hipLaunchKernelGGL(k_sends<true>, dim3(grid), dim3(256), 0, s, gs, gp, st, p, cap, snd, rcv, msg, lost, cnt);
  else
    hipLaunchKernelGGL(k_sends<false>, dim3(grid), dim3(256), 0, s, gs, gp, st, p, cap, snd, rcv, msg, lost, cnt);
  return hipGetLastError();
}

hipError_t launch_drop(const DevState& st, int32_t round, const uint64_t* list, int64_t n, bool check,
                       unsigned long long* hits, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_drop, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, st, round, list, n, check,
                     hits);
  return hipGetLastError();
}

hipError_t launch_rebuild_aw(const DevState& st, int32_t round, int64_t V, hipStream_t s) {
  if (!st.AW[round & 1] || st.W > 64) return hipSuccess;
  hipLaunchKernelGGL(k_rebuild_aw, dim3(grid_tasks((V + 31) >> 5)), dim3(256), 0, s, st, round, V);
  return hipGetLastError();
}

}  // namespace p2pg
