// Gossip fused dense round for narrow rows (W <= 32 words = up to 2048 concurrent
// broadcasts): several peers per wave.
//
// Why: the fused kernel of relay_kernels.hip (k_gossip_fused) maps one peer row to one wave,
// lane = word.  At W = 64 that is one coalesced 512 B row per wave; at W = 8 (one rank's share
// when the 4096 broadcasts of config 4 are split over 8 GPUs) 56 of its 64 lanes idle and every
// peer still costs a whole wave visit, so a step took as long as the W = 64 step (250 vs 294
// ms, profiles/r02/bench_c4_m512_v15.json).  Here a wave takes a BATCH of consecutive peers:
//   lane = (batch peer g, word w), g = lane / WP, w = lane % WP, WP = W rounded up to a power
//   of two, at most 64 / WP peers and at most 64 adjacency slots per batch (or one wider peer);
// so a batch's seen / frontier rows are one contiguous run of memory, its adjacency slots one
// contiguous range of colidx / rev (peers are consecutive), and the per-peer fixed work (row
// offsets, neighbour ids, activity words, the pick loop, the flush) is shared by the batch.
//
// Per batch (same results as k_gossip_fused):
//   1. gather: for every adjacency slot j of the batch (lane = slot, 64 per window) whose
//      neighbour v was active in round r-1 (A bit, churn of round r-1 applied), the owner peer's
//      lanes load E row j (receiver-major: what v pushed to that peer in round r-1; packed when
//      W > PACK_W_MAX_PLAIN: word w at position popcount(AW[v] & below w), else whole) -- the
//      slot index and v's word mask reach the owner's lanes by ds_bpermute;
//   2. dedup against seen, new frontier row, AW mask, A / S bits, counters;
//   3. picks: the new (peer, message) bits are compacted into an LDS list, lanes evaluate
//      Philox + Floyd (gossip_picks_t) and OR the message bit into an LDS table indexed by
//      (batch slot, word); then the flush stores, for every batch slot and every active word
//      of its peer, the table word into the RECEIVER's packed E row of the connection
//      (rev[slot]), zeros included (receivers gather by the sender's AW mask).
// Hubs (deg > HUB_T) are left to the hub kernels, as in k_gossip_fused.
#include "device_util.h"

namespace p2pg {
namespace {

constexpr int GLIST_G = 1024;  // new bits listed per pick pass (a peak-round batch: ~700)
// E-row gathers per lane issued one batch ahead (and per round trip after that)
#ifndef P2PG_GFG
#define P2PG_GFG 6  // c4 A/B (profiles/r03/ab_gfg.txt): W = 8 fused 49.7 -> 47.7 ms, W = 16 97.2 -> 94.1 ms; 8 spills
#endif
constexpr int GFG = P2PG_GFG;

template <int LW>
struct GroupedLds {
  static constexpr int WP = 1 << LW;
  // table slots: 512 (slot, word) masks (4 KB), 64 slots at most; a batch spans at most TS
  // slots (one wider peer: several pick windows), so ~6.5 KB of LDS per wave allows 4 waves
  // per SIMD
  static constexpr int TS = (512 >> LW) < 64 ? (512 >> LW) : 64;
  alignas(8) uint32_t tbl[TS][WP][2];  // (slot, word) mask as two 32-bit halves (LDS atomics)
  uint16_t lst[GLIST_G];               // new bits: lane << 6 | bit
  int32_t off[36];                     // batch peer i -> first slot of its row, batch-relative
  uint32_t swm[64];                    // pick-window slot -> active words of its peer's new row
  uint8_t owner[64];                   // pick-window slot -> batch peer (churn only)
};

__device__ __forceinline__ uint64_t bits_between(int lo, int hi) {  // bits [lo, hi), 0 <= lo, hi <= 64
  const uint64_t below_hi = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
  const uint64_t below_lo = lo >= 64 ? ~0ull : ((1ull << lo) - 1ull);
  return hi > lo ? below_hi & ~below_lo : 0ull;
}

// One batch's registers as it moves through the software pipeline (see the kernel).
struct GStage {
  int b0, n;          // task peers b0 .. b0+n-1 (n = 0: no batch)
  uint32_t rb0, rb1;  // its adjacency slot range (slot ids fit 32 bits: rev[] holds them)
  uint64_t s;         // lane (g, w): seen word
  int32_t v;          // lane = slot of the first 64: neighbour id ...
  uint32_t rv;        // ... the receiver's slot of the connection (rev) ...
  uint32_t aword;     // ... the neighbour's activity word (round r-1) ...
  uint64_t amv;       // ... and its active-word mask
  bool rcv;           // slot exists and its owner peer is processed
};

#ifndef P2PG_GROUPED_WAVES
#define P2PG_GROUPED_WAVES 4  // <= 128 VGPRs
#endif
// PO (push only): the first dense round after an update -- the batch peers are the round's
// active peers, their arrivals are their own frontier rows F[r&1] (dedup, counters, bitmaps were
// done by the update), and only the picks and the flush run (replaces one wave per source with
// 8 of 64 lanes busy at W = 8).
// PL (pull only): the last dense round before the sparse ones -- arrivals gathered from E, dedup,
// frontier rows and bitmaps as in a fused round, no picks and no flush (the round's pushes go by
// row atomics afterwards).  The one-peer-per-wave pull (k_pull1) spends a whole wave visit on
// every peer with 8 of 64 lanes busy at W = 8.
template <bool CHURN, int K, int LW, bool PO = false, bool PL = false>
__global__ __launch_bounds__(256, P2PG_GROUPED_WAVES) void k_gossip_fused_grouped(DevGraph g, DevState st, RoundParams p) {
  using Lds = GroupedLds<LW>;
  // never partitioned and never on a pre-update graph (the engine's dense rounds): the id
  // translation and lost-slot tests fold away
  g.gid = nullptr;
  g.gdeg = g.gpos = nullptr;
  g.gone = nullptr;
  constexpr int WP = Lds::WP;
  constexpr int TS = Lds::TS;
  constexpr int GMAX = (64 >> LW) < 32 ? (64 >> LW) : 32;  // peers per batch
  constexpr int SPI = 64 / WP;                              // flush: slots per instruction
  constexpr int KK = K > 0 ? K : 16;
  __shared__ Lds lds[WPB];
  const int lane = threadIdx.x & 63;
  Lds& L = lds[wave_in_block()];
  const int64_t V = g.V;
  const int W = st.W;
  const int cur = p.round & 1, prv = cur ^ 1;
  const uint64_t* __restrict__ Src = st.E[prv];
  uint64_t* __restrict__ Eo = st.E[cur];
  uint64_t* __restrict__ Fc = st.F[cur];
  const uint32_t* __restrict__ Ap = st.A[prv];
  const uint64_t* __restrict__ AWp = st.AW[prv];
  // packed E rows (sender's active words only, positions from AW) when AW planes exist --
  // W > PACK_W_MAX_PLAIN, i.e. LW >= 4 (the launcher checks it); narrower rows are stored whole,
  // zeros included, so that a receiver needs no random 8 B read of the sender's word mask per
  // connection.  A compile-time fact: one gather path per instance.
  constexpr bool packed = LW > 3;
  static_assert((1 << 3) == PACK_W_MAX_PLAIN, "packed <=> LW > 3 needs PACK_W_MAX_PLAIN == 8");
  const int k = K > 0 ? K : p.fanout;
  const int gl = lane >> LW;        // this lane's batch peer
  const int wl = lane & (WP - 1);   // this lane's word
  const bool wvalid = wl < W;
  const uint32_t below_wl = (1u << wl) - 1u;  // this lane's lower words (wl < 32)
  const uint64_t fm = wvalid ? full_mask(wl, W, st.M) : 0ull;
  const uint64_t gmask = (1ull << WP) - 1ull;
  const int64_t ntasks = (V + 31) >> 5;
  // wave totals in 32 bits (8 fewer scalar registers): a wave of a balanced grid (<= 32 x the
  // resident blocks) covers few tasks -- c4: ~2.4 -- so even 10^9 peers keep its relay / wedge
  // sums (<= tasks x 32 peers x 4096 messages x fanout 16; hubs excluded) far below 2^32
  uint32_t tot[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};

  for (int32_t task = (int32_t)blockIdx.x * WPB + wave_in_block(); task < ntasks;
       task += (int32_t)gridDim.x * WPB) {
    const int64_t u0 = (int64_t)task << 5;
    const uint32_t sat0 = PO ? 0u : st.S[task];
    const int nv = V - u0 < 32 ? (int)(V - u0) : 32;
    uint32_t todo = PO ? st.A[cur][task] : ~sat0;
    if (g.H) todo &= ~g.H[task];  // hubs: k_pull_hub_* and the chunk-item scatter
    if (nv < 32) todo &= (1u << nv) - 1u;
    if (!todo) {
      if (!PO && lane == 0) st.A[cur][task] = 0u;
      continue;
    }
    uint32_t rp = 0;  // lane l <= nv: rowptr[u0 + l] (32-bit slot ids)
    if (lane <= nv) rp = (uint32_t)g.rowptr[u0 + lane];
    uint32_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t aw = 0, sat = sat0;
    uint32_t rest = todo;

    // ---- pipeline stages (software pipeline over the task's batches, as in k_gossip_fused:
    // rows of t+3, activity of t+2, first gathers of t+1 are in flight while t is consumed)
    auto rows = [&](GStage& q) {
      q.n = 0;
      q.rcv = false;
      q.s = 0;
      q.v = 0;
      q.rv = 0;
      if (!rest) return;
      // the batch: <= GMAX consecutive peers and <= TS slots, or one wider peer
      const int b0 = __builtin_ctz(rest);
      const uint32_t rb0 = (uint32_t)__builtin_amdgcn_readlane((int)rp, b0);
      const bool fits = lane > b0 && lane <= b0 + GMAX && lane <= nv && rp - rb0 <= (uint32_t)TS;
      const int cnt = __popcll(__ballot(fits));
      const int n = cnt > 0 ? cnt : 1;
      rest &= (b0 + n >= 32 ? 0u : ~0u << (b0 + n));
      q.b0 = b0;
      q.n = n;
      q.rb0 = rb0;
      q.rb1 = (uint32_t)__builtin_amdgcn_readlane((int)rp, b0 + n);
      const bool mine = gl < n && ((todo >> (b0 + gl)) & 1u);
      // PO: the peer's frontier row (its new receipts) instead of its seen row
      if (mine && wvalid) q.s = ld_once(&(PO ? Fc : st.seen)[(u0 + b0 + gl) * W + wl]);
      // batch peer owning slot rb0 + lane: the number of later row starts at or below it
      // (32-bit offsets relative to the batch; a batch spans <= TS slots or one peer)
      const uint32_t rel = (uint32_t)(rp - rb0);
      int gj = 0;
      for (int i = 1; i < n; ++i)
        gj += (uint32_t)__builtin_amdgcn_readlane((int)rel, b0 + i) <= (uint32_t)lane;
      q.rcv = rb0 + (uint32_t)lane < q.rb1 && ((todo >> (b0 + gj)) & 1u);
      if (q.rcv) {
        q.v = ld_once(&g.colidx[rb0 + (uint32_t)lane]);
        q.rv = ld_once(&g.rev[rb0 + (uint32_t)lane]);
      }
    };
    auto activity = [&](GStage& q) {
      q.aword = 0;
      q.amv = 0;
      if (!PO && q.rcv) {
        q.aword = Ap[q.v >> 5];
        if (packed) q.amv = AWp[q.v];
      }
    };
    // lane (g, w): need = words of peer g still open; the owner's slot range within 64 lanes
    auto need_of = [&](const GStage& q) -> uint64_t {
      const bool mine = gl < q.n && ((todo >> (q.b0 + gl)) & 1u);
      return mine ? (PO ? ~0ull : fm & ~q.s) : 0ull;
    };
    auto my_slots = [&](const GStage& q, uint32_t cb) -> uint64_t {
      const int bi = gl < q.n ? q.b0 + gl : q.b0;
      const int64_t lo = (int64_t)bperm(bi, rp) - (int64_t)cb, hi = (int64_t)bperm(bi + 1, rp) - (int64_t)cb;
      return bits_between(lo < 0 ? 0 : (lo > 64 ? 64 : (int)lo), hi < 0 ? 0 : (hi > 64 ? 64 : (int)hi));
    };
    uint64_t X[GFG];
    auto x_or = [&]() {
      uint64_t o = 0;
#pragma unroll
      for (int qq = 0; qq < GFG; ++qq) o |= X[qq];
      return o;
    };
    // The active slots of one 64-slot window, compacted: lane r holds the r-th active slot's
    // window index (cw_slot) and, packed, its sender's word mask (cw_am); a batch's slots are
    // ordered by owner, so lane (g, w)'s peer owns entries [cw_base, cw_base + cw_cnt).  Gather k
    // of a lane is then one ds_bpermute of entry cw_base + k -- a per-lane 64-bit slot mask
    // (ctz, clear lowest, compare: ~9 VALU per gather) did the same walk before.  One window is
    // live at a time: the first gathers of batch t+1 build it after batch t's last gathers.
    uint32_t cw_slot = 0, cw_am = 0, cw_base4 = 0, cw_cnt = 0;
    auto window = [&](uint64_t am, uint64_t amv, uint64_t ms, bool want) {
      const bool act = (am >> lane) & 1ull;
      const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
      // an inactive lane writes to entry 63, which is read only when all 64 slots are active
      const int dst = (act ? (int)r : 63) << 2;
      cw_slot = (uint32_t)__builtin_amdgcn_ds_permute(dst, lane);
      if constexpr (packed) cw_am = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)amv);
      const uint64_t below = ms & (0ull - ms);  // lowest slot of this lane's peer: entries before it
      cw_base4 = (uint32_t)__popcll(am & (below - 1ull)) << 2;
      cw_cnt = want ? (uint32_t)__popcll(am & ms) : 0u;
    };
    // gathers k0 .. k0 + GFG - 1 of this lane's peer in window cb
    auto gathers = [&](uint32_t cb, uint32_t k0) {
      // the window's first E row (wave-uniform); a gather's offset in the window is < 64 x W
      // words, 32-bit: a scalar base and a 32-bit lane offset per load
      const uint64_t* __restrict__ win = Src + (uint64_t)cb * (uint32_t)W;
#pragma unroll
      for (int qq = 0; qq < GFG; ++qq) {
        const uint32_t k = k0 + (uint32_t)qq;
        const bool ok = k < cw_cnt;
        const int e4 = (int)(cw_base4 + (k << 2));
        const uint32_t idx = (uint32_t)__builtin_amdgcn_ds_bpermute(e4, (int)cw_slot) & 63u;
        bool here = ok;
        uint32_t pos = (uint32_t)wl;
        if constexpr (packed) {
          // the sender's active-word mask: W <= 32 words
          const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(e4, (int)cw_am);
          here = ok && ((a >> wl) & 1u);
          pos = (uint32_t)__popc(a & below_wl);
        }
        // (an int64 slot x width product per lane took two v_mad_u64_u32 and moves per gather)
        const uint32_t ob = (idx * (uint32_t)W + pos) << 3;  // bytes: a scalar-base + lane-offset load
        X[qq] = here ? __builtin_nontemporal_load(
                           reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(win) + ob))
                     : 0ull;
      }
    };
    auto more = [&](uint32_t k0) { return __ballot(k0 < cw_cnt) != 0ull; };
    auto active_slots = [&](const GStage& q, uint32_t cb, int32_t v, bool rcv, uint32_t aword) -> uint64_t {
      bool act = rcv && ((aword >> (v & 31)) & 1u);
      if (CHURN && act) {
        int gj = 0;
        for (int i = 1; i < q.n; ++i) gj += (uint32_t)__builtin_amdgcn_readlane((int)rp, q.b0 + i) <= cb + (uint32_t)lane;
        act = !churn_dropped((uint32_t)(p.round - 1), gidx(g, u0 + q.b0 + gj), gidx(g, v), p.churn_thr,
                             p.cseed_lo, p.cseed_hi);
      }
      return __ballot(act);
    };
    auto first_gathers = [&](GStage& q) {
#pragma unroll
      for (int qq = 0; qq < GFG; ++qq) X[qq] = 0ull;
      cw_cnt = 0;
      if (PO || q.n == 0) return;
      const uint64_t need = need_of(q);
      const uint64_t am = active_slots(q, q.rb0, q.v, q.rcv, q.aword);
      const uint64_t ms = my_slots(q, q.rb0);  // ds_bpermute: evaluated by every lane
      window(am, q.amv, ms, need != 0ull);
      gathers(q.rb0, 0u);
    };

    // ---- the flush of a consumed batch: lane = (slot, word), every active word of the slot's
    // peer into the receiver's packed E row (zeros included: receivers gather by AW mask)
    auto flush = [&](const GStage& q, int32_t p0, int ns) {
      for (int s0 = 0; s0 < ns; s0 += SPI) {
        const int sl = s0 + gl;
        const bool ok = sl < ns && wvalid;
        const uint32_t wmk = ok ? L.swm[sl] : 0u;
        const int js = p0 + sl;  // batch slot
        uint32_t rv = bperm(js & 63, q.rv);
        int32_t tv = CHURN ? (int32_t)bperm(js & 63, (uint32_t)q.v) : 0;
        const int o = CHURN ? (int)L.owner[sl < ns ? sl : 0] : 0;  // churn: the sending peer
        // packed: the sender's active words, in order; else every word of an active sender
        if (packed ? ((wmk >> wl) & 1u) != 0u : (wmk != 0u && wvalid)) {
          if (js >= 64) {  // beyond the registers (one peer wider than 64 slots)
            rv = g.rev[q.rb0 + js];
            if (CHURN) tv = g.colidx[q.rb0 + js];
          }
          uint64_t x = *reinterpret_cast<const uint64_t*>(&L.tbl[sl][wl][0]);
          if (CHURN && x &&
              churn_dropped((uint32_t)p.round, gidx(g, u0 + q.b0 + o), gidx(g, tv), p.churn_thr,
                            p.cseed_lo, p.cseed_hi))
            x = 0ull;
          st_row(Eo + (uint64_t)rv * (uint32_t)W + (packed ? __popc(wmk & below_wl) : wl), x);
          if (x) c[ST_SCATTER] += 1;
        }
      }
    };
    bool pend = false;  // the last consumed batch's flush is deferred to after the next wait
    int pend_ns = 0;

    auto consume = [&](GStage& a, GStage& b, GStage& cc, GStage& d) {
      // 1. arrivals: the first gathers (in flight since the last step) + the rest
      uint64_t acc = x_or();
      const uint64_t need = need_of(a);
      if (PO) acc = a.s;  // the frontier row
      if (!PO) {
        for (uint32_t k0 = GFG; more(k0); k0 += GFG) {  // (the window of a's first gathers)
          gathers(a.rb0, k0);
          acc |= x_or();
        }
        for (uint32_t cb = a.rb0 + 64; cb < a.rb1; cb += 64) {  // one peer wider than 64 slots
          int32_t v = 0;
          uint32_t aword = 0;
          uint64_t amv = 0;
          const bool own = cb + lane < a.rb1 && ((todo >> a.b0) & 1u);
          if (own) {
            v = g.colidx[cb + lane];
            aword = Ap[v >> 5];
            if (packed) amv = AWp[v];
          }
          const uint64_t am = active_slots(a, cb, v, own, aword);
          const uint64_t ms = my_slots(a, cb);
          window(am, amv, ms, need != 0ull);
          for (uint32_t k0 = 0; more(k0); k0 += GFG) {
            gathers(cb, k0);
            acc |= x_or();
          }
        }
      }
      // everything loaded so far has landed: say so explicitly, so that no implicit wait on a
      // younger load (the next batch's gathers) is placed where this batch's data is used
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      if (pend) {
        flush(d, 0, pend_ns);
        pend = false;
      }
      // 2. advance the pipeline before this batch's stores and picks
      first_gathers(b);
      activity(cc);
      rows(d);
      // 3. dedup, frontier row, bitmaps, counters
      const int n = a.n;
      const int bi = gl < n ? a.b0 + gl : a.b0;
      const bool mine = gl < n && ((todo >> bi) & 1u);
      const int64_t u = u0 + bi;
      const uint32_t degg = bperm(bi + 1, rp) - bperm(bi, rp);
      const uint64_t nw = acc & need;
      const uint64_t wm_all = __ballot(nw != 0ull);
      const uint32_t grp = (uint32_t)((wm_all >> (gl * WP)) & gmask);  // my peer's active words
      if (!PO) {
        if (nw) st_frow(&st.seen[u * W + wl], a.s | nw);
        if (mine && grp && wvalid && p.store_f) st_frow(&Fc[u * W + wl], nw);
        if (nw) {
          const uint32_t pc = (uint32_t)__popcll(nw);
          c[ST_NEW] += pc;
          c[ST_RELAYS] += pc * (degg < (uint32_t)k ? degg : (uint32_t)k);
          c[ST_ACTIVE_W] += 1;
          c[ST_WEDGES] += degg;
        }
        if (mine && wl == 0 && grp) {
          if (packed) st.AW[cur][u] = grp;
          c[ST_ACTIVE_V] += 1;
          c[ST_DEG_ACT] += degg;
        }
        aw |= (uint32_t)__ballot(lane < n && ((wm_all >> (lane * WP)) & gmask) != 0u) << a.b0;
        const uint64_t open = __ballot(mine && wvalid && (a.s | nw) != fm);
        const bool done_i = lane < n && ((todo >> (a.b0 + lane)) & 1u) && ((open >> (lane * WP)) & gmask) == 0ull;
        sat |= (uint32_t)__ballot(done_i) << a.b0;
      }
      const uint32_t gi = lane < n ? (uint32_t)((wm_all >> (lane * WP)) & gmask) : 0u;
      if (PL || !wm_all) return;
      // 4. this round's pushes: picks into the (slot, word) table, then the flush
      const int32_t rel = (int32_t)(rp - a.rb0);
      if (lane >= a.b0 && lane <= a.b0 + n) L.off[lane - a.b0] = rel;
      const uint32_t cntb = (uint32_t)__popcll(nw);
      const uint32_t incl = wave_scan_u32(cntb);
      const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      const uint32_t pos0 = incl - cntb;
      const int32_t nslots = (int32_t)(a.rb1 - a.rb0);
      const uint32_t gv_base = (uint32_t)(u0 + a.b0);
      for (int32_t p0 = 0; p0 < nslots; p0 += TS) {
        const int ns = nslots - p0 < TS ? nslots - p0 : TS;
        // the flush's word mask per window slot: its owner's new words
        int o = 0;
        for (int i = 1; i < n; ++i) o += __builtin_amdgcn_readlane(rel, a.b0 + i) <= p0 + lane;
        const uint32_t swm = bperm(o, gi);
        if (lane < ns) {
          L.swm[lane] = swm;
          if (CHURN) L.owner[lane] = (uint8_t)o;
        }
        for (int e = lane; e < ns * WP; e += 64)  // (slot, word) masks, one 64-bit write each
          reinterpret_cast<uint64_t*>(&L.tbl[0][0][0])[e] = 0ull;
        for (uint32_t lb = 0; lb < total; lb += GLIST_G) {
          const uint32_t ne = total - lb < (uint32_t)GLIST_G ? total - lb : (uint32_t)GLIST_G;
          uint32_t li = pos0 - lb;
          for (uint32_t h = (uint32_t)nw; h; h &= h - 1u, ++li)
            if (li < ne) L.lst[li] = (uint16_t)(((uint32_t)lane << 6) | (uint32_t)__builtin_ctz(h));
          for (uint32_t h = (uint32_t)(nw >> 32); h; h &= h - 1u, ++li)
            if (li < ne) L.lst[li] = (uint16_t)(((uint32_t)lane << 6) | 32u | (uint32_t)__builtin_ctz(h));
          wave_lds_sync();
          // strided: lane l takes entries l*nbat ..: consecutive entries are one word's bits
          const uint32_t nbat = (ne + 63) >> 6;
          const uint32_t i0 = (uint32_t)lane * nbat;
          const uint32_t my = i0 < ne ? (ne - i0 < nbat ? ne - i0 : nbat) : 0u;
          for (uint32_t bb = 0; bb < my; ++bb) {
            const uint32_t e = L.lst[i0 + bb];
            const uint32_t le = e >> 6, bit = e & 63u;
            const int gq = (int)(le >> LW), wq = (int)(le & (WP - 1));
            const int32_t oq = L.off[gq];
            const uint32_t dq = (uint32_t)(L.off[gq + 1] - oq);
            const uint32_t mb = 1u << (bit & 31u);
            uint32_t* const col = &L.tbl[0][wq][bit >> 5];
            const int32_t base = oq - p0;
            if (dq <= (uint32_t)k) {  // every connection (node.py:114-120 per target)
              for (uint32_t q = 0; q < dq; ++q)
                if ((uint32_t)(base + (int32_t)q) < (uint32_t)ns) atomicOr(col + (base + (int32_t)q) * (WP * 2), mb);
            } else {
              uint32_t pk[KK];
              const uint32_t mg = p.msg_base + (uint32_t)wq * 64u + bit;
              if constexpr (K > 0)
                gossip_picks_t<K>((uint32_t)p.round, gidx(g, (int64_t)gv_base + gq), mg, dq, p.gseed_lo,
                                  p.gseed_hi, pk);
              else
                gossip_picks((uint32_t)p.round, gidx(g, (int64_t)gv_base + gq), mg, dq, k, p.gseed_lo,
                             p.gseed_hi, pk);
#pragma unroll
              for (int q = 0; q < KK; ++q) {
                if (q >= k) break;
                const int32_t sl = base + (int32_t)pk[q];
                if ((uint32_t)sl < (uint32_t)ns) atomicOr(col + sl * (WP * 2), mb);
              }
            }
          }
          wave_lds_sync();
        }
        if (nslots <= TS) {  // one window: the flush leaves after the next batch's wait
          pend = true;
          pend_ns = ns;
        } else {
          flush(a, p0, ns);
          wave_lds_sync();
        }
      }
    };

    GStage sA, sB, sC, sD;
    rows(sA);
    rows(sB);
    activity(sA);
    first_gathers(sA);
    activity(sB);
    rows(sC);
    sD.n = 0;
    // the last consumed batch's deferred flush has no next wait to follow: it leaves here
    auto last = [&](const GStage& q) {
      if (pend) flush(q, 0, pend_ns);
      pend = false;
    };
    for (;;) {  // four stages rotate by unrolling (a register copy would wait for its loads)
      consume(sA, sB, sC, sD);
      if (sB.n == 0) { last(sA); break; }
      consume(sB, sC, sD, sA);
      if (sC.n == 0) { last(sB); break; }
      consume(sC, sD, sA, sB);
      if (sD.n == 0) { last(sC); break; }
      consume(sD, sA, sB, sC);
      if (sA.n == 0) { last(sD); break; }
    }
    wave_lds_sync();
    if (!PO && lane == 0) {
      st.A[cur][task] = aw;
      if (sat != sat0) st.S[task] = sat;
    }
#pragma unroll
    for (int q = 0; q < STAT_N; ++q) tot[q] += wave_reduce_u32<false>(c[q]);
  }
  if (lane == 0) {
    unsigned long long* shard = st.stats + (blockIdx.x & (STAT_SHARDS - 1)) * STAT_N;
#pragma unroll
    for (int q = 0; q < STAT_N; ++q)
      if (tot[q]) atomicAdd(shard + q, (unsigned long long)tot[q]);
  }
}

template <bool CH, int KT, bool PO = false, bool PL = false>
hipError_t launch_lw(int lw, const DevGraph& g, const DevState& st, const RoundParams& p, hipStream_t s) {
  const int64_t ntasks = (g.V + 31) >> 5;
#define P2PG_GROUPED(LWV)                                                                    \
  hipLaunchKernelGGL((k_gossip_fused_grouped<CH, KT, LWV, PO, PL>),                        \
                     dim3(balanced_grid(k_gossip_fused_grouped<CH, KT, LWV, PO, PL>, ntasks)), dim3(256), \
                     0, s, g, st, p)
  switch (lw) {
    case 0: P2PG_GROUPED(0); break;
    case 1: P2PG_GROUPED(1); break;
    case 2: P2PG_GROUPED(2); break;
    case 3: P2PG_GROUPED(3); break;
    case 4: P2PG_GROUPED(4); break;
    default: P2PG_GROUPED(5); break;
  }
#undef P2PG_GROUPED
  return hipGetLastError();
}

}  // namespace

// The instances' packed form is LW > 3: it must agree with the state's AW planes.
static bool packed_ok(const DevState& st, int lw, int prv) {
  return (lw > 3) == (st.AW[prv] != nullptr);
}

hipError_t launch_gossip_fused_grouped(const DevGraph& g, const DevState& st, const RoundParams& p,
                                       hipStream_t s) {
  if (st.W > 32 || st.W < 1) return hipErrorInvalidValue;
  int lw = 0;
  while ((1 << lw) < st.W) ++lw;
  if (!packed_ok(st, lw, (p.round & 1) ^ 1)) return hipErrorInvalidValue;
  const bool ch = p.churn_thr != 0;
  if (p.fanout == 3) return ch ? launch_lw<true, 3>(lw, g, st, p, s) : launch_lw<false, 3>(lw, g, st, p, s);
  return ch ? launch_lw<true, 0>(lw, g, st, p, s) : launch_lw<false, 0>(lw, g, st, p, s);
}

hipError_t launch_gossip_push_grouped(const DevGraph& g, const DevState& st, const RoundParams& p,
                                      hipStream_t s) {
  if (st.W > GROUPED_W_MAX || st.W < 1) return hipErrorInvalidValue;
  int lw = 0;
  while ((1 << lw) < st.W) ++lw;
  if (!packed_ok(st, lw, p.round & 1)) return hipErrorInvalidValue;  // (PO: the round's own rows)
  const bool ch = p.churn_thr != 0;
  if (p.fanout == 3)
    return ch ? launch_lw<true, 3, true>(lw, g, st, p, s) : launch_lw<false, 3, true>(lw, g, st, p, s);
  return ch ? launch_lw<true, 0, true>(lw, g, st, p, s) : launch_lw<false, 0, true>(lw, g, st, p, s);
}

hipError_t launch_gossip_pull_grouped(const DevGraph& g, const DevState& st, const RoundParams& p,
                                      hipStream_t s) {
  if (st.W > GROUPED_PULL_W_MAX || st.W < 1) return hipErrorInvalidValue;
  int lw = 0;
  while ((1 << lw) < st.W) ++lw;
  if (!packed_ok(st, lw, (p.round & 1) ^ 1)) return hipErrorInvalidValue;
  // (no picks: the fanout template argument is irrelevant)
  return p.churn_thr != 0 ? launch_lw<true, 0, false, true>(lw, g, st, p, s)
                          : launch_lw<false, 0, false, true>(lw, g, st, p, s);
}

}  // namespace p2pg
