// Host side of the relay engine: the C-ABI declared in include/p2pgpu.h.
//
// One engine = one GPU = one simulated peer graph resident in HBM.  Per round it launches a
// handful of HIP kernels (relay_kernels.hip) on one stream and copies back 8 shards x 8
// counters; nothing else crosses PCIe inside a run.
//
// Round schedule (r = round index; pushes made in round r arrive in round r+1):
//   r = 0          seed: F[0], seen, A[0] <- source bits    (Node.send_to_nodes at the origin,
//                                                            p2pnetwork/node.py:106-112)
//   flood  r >= 1  pull:   F[r&1], A[r&1], seen <- OR of active neighbours' F[(r-1)&1]
//   gossip r >= 1  update: F[r&1], A[r&1], seen <- next[r&1] & ~seen  (T[r&1] = touched rows)
//   gossip r >= 0  scatter: next[(r+1)&1], T[(r+1)&1] |= k Philox picks of every F[r&1] bit
//                  (sparse rounds), or E[r&1] per-connection masks (dense rounds; the next
//                  round pulls them; a dense round after a dense round runs pull + scatter
//                  as one fused pass, k_gossip_fused)
//   record         hop/parent planes for the bits of F[r&1]   (P2PG_FLAG_RECORD only)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/p2pgpu.h"
#include "internal.h"

using namespace p2pg;

// round 0's counters (seed_stats)
struct SeedStats {
  bool ok = false;
  uint64_t nw = 0, relays = 0, av = 0, aw = 0, wedge = 0, degact = 0;
};

struct p2pg_engine {
  p2pg_config cfg{};
  std::string err;
  int64_t V = 0, nnz = 0;
  int64_t v_conn = 0;          // peers with >= 1 connection: the ones a round can make active
                               // (the dense-round test compares active peers with these, so
                               // isolated peers do not keep a run sparse)
  int32_t M = 0, W = 0;
  std::vector<int64_t> h_rowptr;
  std::vector<int32_t> h_colidx;  // host copy of the adjacency (topology updates, snapshots)
  std::vector<int32_t> h_src;
  // device
  int64_t* d_rowptr = nullptr;
  int32_t* d_colidx = nullptr;
  int64_t* d_hub = nullptr;
  int64_t n_hub = 0;
  int64_t* d_hub_big = nullptr;  // the chunk items of sources with deg > HUB_T (fused rounds)
  int64_t n_hub_big = 0;
  int32_t* d_wide_big = nullptr;  // sources with deg > HUB_T (fused rounds' hub pushes)
  int64_t n_wide_big = 0;
  uint32_t* d_rev = nullptr;   // gossip: reverse edge slots
  // pull hub split (deg > HUB_T)
  uint32_t* d_H = nullptr;
  int64_t* d_hub_items = nullptr;
  int32_t* d_hubs = nullptr;
  int64_t* d_hub_begin = nullptr;
  uint64_t* d_partial = nullptr;
  HubPlan hp{};
  // vertex-partitioned runs
  int32_t* d_gid = nullptr;
  std::vector<int32_t> h_gid;
  int32_t* d_gdeg = nullptr;          // ghost senders' global degrees (p2pg_set_ghost_senders)
  int32_t* d_gpos = nullptr;          // per local slot: position in the ghost neighbour's row
  int32_t* d_send = nullptr;
  int32_t* d_recv = nullptr;
  int64_t n_send = 0, n_recv = 0;
  uint32_t* d_border = nullptr;       // owned peers with a ghost neighbour (phase 1 of a round)
  std::vector<int64_t> send_seg, recv_seg;  // list offsets per rank (p2pg_set_exchange_segments)
  int64_t* d_send_seg = nullptr;
  int64_t* d_recv_seg = nullptr;
  unsigned long long* d_seg_cnt = nullptr;  // live rows per destination (pack_live)
  unsigned long long* h_seg_cnt = nullptr;  // pinned
  // p2pg_set_exchange_buffer: every round packs its live rows of this plane into this buffer
  // right after its kernels, and the counts come back with the round counters (one host
  // synchronisation per round); pack_live then only hands them over
  void* auto_buf = nullptr;
  int32_t auto_plane = -1;
  int32_t auto_round = -1;           // the round whose records auto_buf / auto_cnt hold
  int64_t auto_cnt[P2PG_MAX_RANKS] = {0};  // their counts per destination (h_seg_cnt is reused
                                           // by explicit packs of the other plane)
  bool begun = false;                 // p2pg_step_begin ran this round's phase 0
  bool last_push_e = false;    // gossip: pushes of the previous round went to E (dense)
  double e_thresh = 0.06;      // store-mode when active words >= thresh * active rows * W;
  double e_thresh_env = -1.0;  // P2PG_E_THRESH (>= 0) or by the current row width (alloc_state)
                               // (c4 A/B, interleaved runs: 0.04 320.4 ms vs 0.1 324.3 ms, round 1;
                               // with the lane-parallel sparse push (round 2) W = 64: 0.04 / 0.06 /
                               // 0.08 -> 278.4 / 275.5 / 275.2 ms, W = 8: 89.1 / 89.4 / 89.5 ms)
  double v_thresh = 0.3;       // ... and active rows >= v_thresh * v_conn (by row width, alloc_state;
  double v_thresh_env = -1.0;  // P2PG_V_THRESH overrides): a dense round visits every
                               // unsaturated peer, a sparse one only the pushed-to rows (narrow
                               // rows: word density alone is high whenever anything is active)
  int push_mode = 0;           // 0 auto, 1 always row atomics, 2 always edge stores
  bool fused = true;           // dense rounds after dense rounds: one pull+scatter pass
  bool wide_atomic = true;     // fused rounds: hub pushes by atomics (P2PG_WIDE_ATOMIC=0: one
                               // wave per 16-connection chunk item)
  int push_dedup = -1;         // sparse pushes drop seen bits: -1 in the decay phase, 0 never,
                               // 1 always (P2PG_PUSH_DEDUP)
  bool sparse_lp = true;       // sparse rounds: lane-parallel scatter (relay_sparse.hip) when
                               // the rows allow it; P2PG_SPARSE_LP=0 keeps the per-source one
  bool skip_frontier = false;  // p2pg_run, not its last two allowed rounds: fused rounds may skip F
  bool partial_f = true;       // ... and updates / the last dense pull write its nonzero words
                               // only (P2PG_PARTIAL_F=0: whole rows, A/B)
  bool frontier_kept = true;   // F[(round-1)&1] holds the last round's first receipts
  bool frontier_kept_prev = true;  // ... and F[round&1] the round before (delivery parents)
  uint64_t prev_aw = 0, prev_av = 0;  // active words / rows of the previous round
  uint64_t last_new = 0;       // first receipts of the last round run
  uint64_t prev2_aw = 0, prev2_av = 0, prev2_new = 0;  // the same, one round earlier
  uint64_t prev_sw = 0;        // distinct masks pushed in the last round (>= the next frontier's
                               // nonzero words: each of them received at least one)
  bool saw_dense = false;      // a round of this run pushed into E (the dense phase has begun)
  bool decay_pred = true;      // still_dense shrinks the counters in the decay phase
                               // (P2PG_DECAY_PRED=0: the last round's counters as they are)
  int update_push = -1;        // the first dense round after a sparse one: its update and its
                               // E pushes in one pass (launch_gossip_update_push) -- -1 when the
                               // round is predicted dense (predict_dense), 0 never, 1 whenever
                               // the rows allow it (P2PG_UPDATE_PUSH)
  int32_t* d_src = nullptr;
  DevState st{};
  size_t plane_bytes = 0, bm_bytes = 0;
  unsigned long long* h_stats = nullptr;  // pinned
  // The round counters accumulate on the device across rounds (no per-round clearing launch): a
  // round's counters are the difference to stats_base, the copy read at the end of the round
  // before.  stats_clear: the device counters must be zeroed first (new state, reset, restore, or
  // an out-of-round launch that counted: a topology update's re-push, a snapshot's materialize)
  unsigned long long stats_base[STAT_N * STAT_SHARDS] = {0};
  bool stats_clear = true;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipEvent_t ev_sync = nullptr;  // round_sync's marker (no timing)
  bool spin = false;             // round_sync polls the marker instead of blocking (P2PG_SPIN)
  // per-launch timing events: recorded around each launch, resolved after the round's stream
  // sync (no extra host synchronisation inside a round)
  std::vector<hipEvent_t> ev_pool;
  std::vector<int> ev_cls;  // class of pending pair i (events 2i, 2i+1)
  uint32_t timed_mask = (1u << P2PG_KCLASS_N) - 1u;  // classes whose launches get events
  double kms[P2PG_KCLASS_N] = {0};
  int64_t klaunch[P2PG_KCLASS_N] = {0};
  int32_t round = 0;
  bool done = false;
  bool have_state = false;
  std::string failed;           // non-empty: the device state is inconsistent (a batched round's
                                // push list overflowed); every step / run refuses until a reset
  // after a topology update: the graph the in-flight messages were sent on and its removed
  // slots, kept for the parents (record / deliveries) of the round that receives them
  int64_t* d_rowptr_arr = nullptr;
  int32_t* d_colidx_arr = nullptr;
  uint8_t* d_gone = nullptr;
  int32_t arr_round = -1;       // the round whose arrivals travelled on that graph
  bool consume_next = false;    // the next round consumes materialized rows (update kernel)
  uint64_t total_relays = 0;    // relays since the last reset (= sum of message_count_send)
  // sparse-round scatter (relay_sparse.hip): the (peer, word) list of a frontier; its fill
  // count lives in the stats buffer, slot STAT_COUNT
  uint64_t* d_wlist = nullptr;
  int64_t wlist_cap = 0;
  uint8_t* d_touched = nullptr;  // one byte per peer (V rounded up to 32), zero between launches
  uint32_t* d_chunk_cnt = nullptr;  // per list chunk: pairs, and their offsets
  uint64_t* d_chunk_off = nullptr;
  bool wlist_check = false;     // a sparse scatter ran this round: check its count after it
  // p2pg_run's decay-phase batches: round counters of up to BATCH_MAX rounds (one slot each)
  unsigned long long* d_bstats = nullptr;
  unsigned long long* h_bstats = nullptr;  // pinned
  int batch_rounds = -1;        // P2PG_RUN_BATCH (rounds per host synchronisation in the decay
                                // phase; 1 = none), -1 = the default
  // Double-buffered seen plane: a reset swaps in the spare (zeroed earlier) and zeroes the plane
  // it replaces on a side stream, behind the work already queued -- the zeroing overlaps the next
  // run's first rounds (latency-bound sparse rounds) instead of leading it.  P2PG_SEEN_SPARE=0,
  // a plane above 1/16 of the device or a failed allocation: the reset zeroes seen in stream
  // order (spare_ready).
  bool seen_spare_on = true;    // P2PG_SEEN_SPARE (for good)
  bool seen_spare_off = false;  // the current plane size / free memory ruled it out (re-examined
                                // when the state is allocated again, alloc_state)
  uint64_t* seen_spare = nullptr;
  bool spare_pending = false;   // a zeroing of seen_spare is queued on `side` (ev_spare marks it)
  hipStream_t side = nullptr;
  hipEvent_t ev_spare = nullptr, ev_main = nullptr;
  SeedStats seed;               // round 0's counters (seed_stats), valid for these sources / rows
  // the arrivals of the next round (p2pg_round_stats.received): the last round's sends
  // (send_to_node calls, less the relays p2pg_drop_relays withdrew) and how many of them are
  // lost -- to churn (counted after every round of a churn run: cnt_lost) or to a connection a
  // topology update removed (counted by p2pg_update_edges)
  uint64_t sent_last = 0, lost_last = 0;
  unsigned long long* d_cnt2 = nullptr;  // k_sends counters [2] (device) / pinned copy
  unsigned long long* h_cnt2 = nullptr;
};

namespace {

// stats buffer: STAT_N x STAT_SHARDS round counters, then the sparse scatter's list count
constexpr int STAT_COUNT = STAT_N * STAT_SHARDS;
constexpr size_t STAT_BYTES = sizeof(unsigned long long) * (STAT_COUNT + 1);

int fail(p2pg_engine* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  set_global_error(msg);
  return code;
}

#define HIPCHK(e, x)                                                                     \
  do {                                                                                   \
    hipError_t _r = (x);                                                                 \
    if (_r != hipSuccess)                                                                \
      return fail(e, P2PG_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(_r));      \
  } while (0)

template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

void free_state(p2pg_engine* e) {
  dfree(e->d_cnt2);
  if (e->h_cnt2) (void)hipHostFree(e->h_cnt2);
  e->h_cnt2 = nullptr;
  DevState& s = e->st;
  dfree(s.seen);
  if (e->seen_spare) {
    if (e->spare_pending) (void)hipStreamSynchronize(e->side);
    dfree(e->seen_spare);
  }
  e->spare_pending = false;
  for (int i = 0; i < 2; ++i) {
    dfree(s.F[i]);
    dfree(s.next[i]);
    dfree(s.A[i]);
    dfree(s.T[i]);
  }
  dfree(s.S);
  dfree(s.hop);
  dfree(s.parent);
  if (s.E[1] == s.E[0]) s.E[1] = nullptr;
  for (int i = 0; i < 2; ++i) dfree(s.E[i]);
  for (int i = 0; i < 2; ++i) dfree(s.AW[i]);
  dfree(s.stats);
  dfree(e->d_wlist);
  e->wlist_cap = 0;
  dfree(e->d_touched);
  dfree(e->d_chunk_cnt);
  dfree(e->d_chunk_off);
#ifdef P2PG_PROF
  if (s.prof) {
    unsigned long long h[16];
    if (hipMemcpy(h, s.prof, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess) {
      fprintf(stderr, "P2PG_PROF");
      for (int i = 0; i < 16; ++i) fprintf(stderr, " %llu", h[i]);
      fprintf(stderr, "\n");
    }
  }
  dfree(s.prof);
#endif
  dfree(e->d_src);
  e->have_state = false;
}

void free_arr(p2pg_engine* e) {
  dfree(e->d_rowptr_arr);
  dfree(e->d_colidx_arr);
  dfree(e->d_gone);
  e->arr_round = -1;
}

// the topology arrays only (rows, reverse slots, hub lists / plans)
void free_topology(p2pg_engine* e) {
  dfree(e->d_rowptr);
  dfree(e->d_colidx);
  dfree(e->d_hub);
  dfree(e->d_hub_big);
  dfree(e->d_wide_big);
  dfree(e->d_rev);
  dfree(e->d_H);
  dfree(e->d_hub_items);
  dfree(e->d_hubs);
  dfree(e->d_hub_begin);
  dfree(e->d_partial);
  e->hp = HubPlan{};
  e->n_hub = 0;
  e->n_hub_big = 0;
  e->n_wide_big = 0;
}

void free_graph(p2pg_engine* e) {
  free_arr(e);
  dfree(e->d_rowptr);
  dfree(e->d_colidx);
  dfree(e->d_hub);
  dfree(e->d_hub_big);
  dfree(e->d_wide_big);
  dfree(e->d_rev);
  dfree(e->d_H);
  dfree(e->d_hub_items);
  dfree(e->d_hubs);
  dfree(e->d_hub_begin);
  dfree(e->d_partial);
  dfree(e->d_gid);
  dfree(e->d_gdeg);
  dfree(e->d_gpos);
  dfree(e->d_send);
  dfree(e->d_recv);
  dfree(e->d_border);
  dfree(e->d_send_seg);
  dfree(e->d_recv_seg);
  dfree(e->d_seg_cnt);
  if (e->h_seg_cnt) (void)hipHostFree(e->h_seg_cnt);
  e->h_seg_cnt = nullptr;
  e->auto_buf = nullptr;
  e->auto_plane = e->auto_round = -1;
  e->send_seg.clear();
  e->recv_seg.clear();
  e->h_gid.clear();
  e->n_send = e->n_recv = 0;
  e->hp = HubPlan{};
  e->n_hub = 0;
  e->n_hub_big = 0;
  e->n_wide_big = 0;
}

RoundParams params(const p2pg_engine* e) {
  RoundParams p{};
  p.round = e->round;
  p.mode = e->cfg.mode;
  p.fanout = e->cfg.fanout;
  p.msg_base = e->cfg.msg_id_base;
  p.gseed_lo = (uint32_t)e->cfg.gossip_seed;
  p.gseed_hi = (uint32_t)(e->cfg.gossip_seed >> 32);
  p.churn_thr = e->cfg.churn_threshold;
  p.cseed_lo = (uint32_t)e->cfg.churn_seed;
  p.cseed_hi = (uint32_t)(e->cfg.churn_seed >> 32);
  p.border = nullptr;
  p.phase = -1;
  p.store_f = 1;
  p.dedup_push = 0;
  return p;
}

DevGraph graph(const p2pg_engine* e) {
  return DevGraph{e->d_rowptr, e->d_colidx, e->d_rev, e->d_H, e->d_gid, nullptr, e->V,
                  e->d_gdeg, e->d_gpos};
}

// The graph round r's arrivals travelled on: the pre-update graph (with its removed slots) for
// the round right after a topology update, else the current one.
DevGraph graph_for_arrivals(const p2pg_engine* e, int32_t r) {
  if (r == e->arr_round && e->d_rowptr_arr)
    return DevGraph{e->d_rowptr_arr, e->d_colidx_arr, nullptr, nullptr, e->d_gid, e->d_gone, e->V,
                    nullptr, nullptr};
  return graph(e);
}

// The host's wait for a round's counters (everything enqueued on the engine's stream so far):
// a blocking stream synchronisation, or -- P2PG_SPIN -- a marker event polled in a loop, which
// trades a spinning host thread for the wake-up latency of a blocking wait (the GPU idles
// between a round's counter copy and the next round's first launch for as long as the host takes
// to notice).
hipError_t round_sync(p2pg_engine* e) {
  if (!e->spin) return hipStreamSynchronize(e->stream);
  hipError_t r = hipEventRecord(e->ev_sync, e->stream);
  if (r != hipSuccess) return r;
  while ((r = hipEventQuery(e->ev_sync)) == hipErrorNotReady) {
  }
  return r;
}

// Timed launch: kernel class cls in [0, P2PG_KCLASS_N) (see include/p2pgpu.h).
template <class F>
int timed(p2pg_engine* e, int cls, F&& launch) {
  const bool timing = (e->cfg.flags & P2PG_FLAG_TIMING) != 0 && ((e->timed_mask >> cls) & 1u);
  size_t slot = 0;
  if (timing) {
    slot = e->ev_cls.size();
    while (e->ev_pool.size() < 2 * (slot + 1)) {
      hipEvent_t ev;
      HIPCHK(e, hipEventCreate(&ev));
      e->ev_pool.push_back(ev);
    }
    HIPCHK(e, hipEventRecord(e->ev_pool[2 * slot], e->stream));
  }
  hipError_t r = launch();
  if (r != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(r));
  if (timing) {
    HIPCHK(e, hipEventRecord(e->ev_pool[2 * slot + 1], e->stream));
    e->ev_cls.push_back(cls);
  }
  e->klaunch[cls] += 1;
  return P2PG_OK;
}

// After a stream sync: fold the pending launch timings into the per-class sums.
int resolve_timings(p2pg_engine* e) {
  for (size_t i = 0; i < e->ev_cls.size(); ++i) {
    float ms = 0.f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev_pool[2 * i], e->ev_pool[2 * i + 1]));
    e->kms[e->ev_cls[i]] += ms;
  }
  e->ev_cls.clear();
  return P2PG_OK;
}

// Can round p's row-atomic push run lane-parallel (relay_sparse.hip)?
bool sparse_scatter_on(const p2pg_engine* e) {
  return e->sparse_lp && gossip_scatter_sparse_supported(e->st);
}

// Buffers of the lane-parallel pushes, grown on demand: a (peer, word) list of >= need entries,
// its chunk counts / offsets, the touched bytes.  Its fill count goes to the stats slot
// STAT_COUNT and is checked after the round (check_scatter_list).
hipError_t sparse_bufs(p2pg_engine* e, int64_t need, SparseBufs& b) {
  need = need > 0 ? need : 1;
  if (need > e->wlist_cap) {
    dfree(e->d_wlist);
    e->wlist_cap = 0;
    const int64_t cap = need + need / 4 + 4096;  // grows by steps, not per round
    hipError_t r = hipMalloc((void**)&e->d_wlist, sizeof(uint64_t) * (size_t)cap);
    if (r != hipSuccess) return r;
    e->wlist_cap = cap;
  }
  if (!e->d_touched) {
    const size_t tb = (size_t)((e->V + 31) >> 5) << 5;
    const size_t nc = ((size_t)sparse_chunks(e->V) + 8) & ~(size_t)7;  // 16 B loads
    hipError_t r = hipMalloc((void**)&e->d_touched, tb ? tb : 32);
    if (r == hipSuccess) r = hipMemsetAsync(e->d_touched, 0, tb ? tb : 32, e->stream);
    if (r == hipSuccess) r = hipMalloc((void**)&e->d_chunk_cnt, sizeof(uint32_t) * nc);
    if (r == hipSuccess) r = hipMalloc((void**)&e->d_chunk_off, sizeof(uint64_t) * nc);
    if (r != hipSuccess) return r;
  }
  e->wlist_check = true;
  b = SparseBufs{e->d_wlist, e->wlist_cap, e->st.stats + STAT_COUNT, e->d_chunk_cnt,
                 e->d_chunk_off, e->d_touched};
  return hipSuccess;
}

// Row-atomic push of the frontier of round p.round over g: lane-parallel when the rows allow it
// (n_words = that frontier's nonzero words, which sizes the (peer, word) list), else per source.
hipError_t launch_scatter_atomic(p2pg_engine* e, const DevGraph& g, const RoundParams& p,
                                 uint64_t n_words) {
  DevState& s = e->st;
  if (!sparse_scatter_on(e))
    return launch_gossip_scatter(g, s, p, e->d_hub, e->n_hub, false, e->stream);
  SparseBufs b;
  hipError_t r = sparse_bufs(e, (int64_t)n_words, b);
  if (r != hipSuccess) return r;
  return launch_gossip_scatter_sparse(g, s, p, (int64_t)n_words, b, e->stream);
}

// Can the fused rounds' hub pushes run by atomics (launch_wide_push_e)?
bool wide_atomic_on(const p2pg_engine* e) {
  return e->wide_atomic && e->W <= 64 && (e->W <= PACK_W_MAX_PLAIN || e->st.AW[0]);
}

// Will the pushes of round e->round (a round after a sparse one, before its update ran) be dense
// by the rule the engine applies to its own stats (use_e below)?  Rising phase only: active words
// grow by the last round's factor and inactive peers shrink by it, with a 15 % margin on the word
// test.  On config 4's recorded rounds at 512 / 1024 / 2048 / 4096 broadcasts this names exactly
// the first dense round at W = 32 / 64 and none at W <= 16 (no false positive).  A wrong guess
// changes the push form of one round, never a result.
bool predict_dense(const p2pg_engine* e) {
  if (e->prev2_aw == 0 || e->prev2_av == 0 || e->last_new <= e->prev2_new) return false;
  const double V = (double)e->v_conn;
  const double in1 = V - (double)e->prev_av, in2 = V - (double)e->prev2_av;
  if (in2 <= 0.0) return false;
  const double est_av = V - in1 * (in1 / in2);
  const double est_aw = (double)e->prev_aw * ((double)e->prev_aw / (double)e->prev2_aw);
  return est_av > 0.0 && est_aw >= 1.15 * e->e_thresh * est_av * (double)e->W &&
         est_av >= e->v_thresh * V;
}

// Will this round's pushes go by row atomics whatever its counters say?  Then the push is
// launched without reading them first (one host synchronisation per round instead of two): in
// the decay phase (after the dense rounds, receipts shrinking) and while the rising frontier is
// far below the dense-round thresholds (active peers, grown twice by the last growth factor, under
// half of v_thresh * v_conn).  Only the push form depends on it, never a result.
bool clearly_sparse(const p2pg_engine* e) {
  if (e->round == 0) return false;  // (origination: the counters are the host's)
  // a bound, not a guess: every active peer of this round received at least one of the masks
  // pushed in the last one (prev_sw), and a dense round needs v_thresh * v_conn active peers
  // (c4: rounds 5 and 6, whose frontiers grow too fast for the guess below)
  if (e->prev_sw > 0 && (double)e->prev_sw < e->v_thresh * (double)e->v_conn) return true;
  if (e->saw_dense) return e->last_new < e->prev2_new;
  if (e->prev_av == 0) return true;  // nothing arrives: an empty round
  const double grow = e->prev2_av ? std::max(1.0, (double)e->prev_av / (double)e->prev2_av) : 64.0;
  return (double)e->prev_av * grow * grow < 0.5 * e->v_thresh * (double)e->v_conn;
}

// A dense round follows a dense round if the frontier it will push is still dense by the rule
// the engine applies to its own counters (use_e in p2pg_step).  The counters are those of the
// round before; in the decay phase (receipts shrinking) they are first shrunk by their last
// factor, so the last dense round is not one round late (c4: round 24's 3.0e7 active words are
// below 0.06 x 8.2e6 peers x 64, while round 23's were above).  Only the push form depends on
// it, never a result.
bool still_dense(const p2pg_engine* e) {
  double aw = (double)e->prev_aw, av = (double)e->prev_av;
  if (e->decay_pred && e->saw_dense && e->last_new < e->prev2_new && e->prev2_aw && e->prev2_av) {
    aw *= aw / (double)e->prev2_aw;
    av *= av / (double)e->prev2_av;
  }
  return av > 0.0 && aw >= e->e_thresh * av * (double)e->W && av >= e->v_thresh * (double)e->v_conn;
}

// Inside p2pg_run (not its last two allowed rounds, no hop/parent records): may this round's update
// / last dense pull write only the nonzero words of its frontier rows (RoundParams::store_f == 2)?
// Packed rows only (16 < W <= 64: AW planes, one peer per wave), not on a partitioned rank.  A
// whole 512 B row write per active peer was ~40 % of the sparse update's bytes; the words are
// read back only through the AW mask (sparse push list, push-only pass, per-source scatter).
bool partial_frontier(const p2pg_engine* e, bool skip) {
  return skip && !e->st.hop && e->st.AW[0] && e->W > GROUPED_W_MAX && e->W <= 64 && !e->d_gid &&
         e->partial_f;
}

// A fused dense round (pull of E[(r-1)&1] + pushes into E[r&1]) and its hub pushes.
hipError_t launch_fused_round(p2pg_engine* e, const DevGraph& g, const RoundParams& p) {
  DevState& s = e->st;
  if (e->d_gid) {  // the exchanged row pushes it ORed in are cleared after the pass
    hipError_t r = launch_gossip_fused(g, s, p, e->hp, nullptr, 0, true, e->stream);
    return r != hipSuccess ? r : launch_clear_arrivals(s, p.round, e->V, e->stream);
  }
  const bool wa = wide_atomic_on(e);
  hipError_t r = launch_gossip_fused(g, s, p, e->hp, e->d_hub_big, e->n_hub_big, wa, e->stream);
  if (r != hipSuccess || !wa) return r;
  return launch_wide_push_e(g, s, p, e->d_hub_big, e->n_hub_big, e->d_wide_big, e->n_wide_big,
                            e->stream);
}

// Can this vertex-partitioned rank (global ids set) take the dense rounds (E pushes, fused and
// pull-only passes in their PART form, relay_kernels.hip)?  Packed rows over 16 < W <= 64 and
// two E planes; otherwise its gossip pushes go by row atomics only.
bool part_dense(const p2pg_engine* e) {
  const DevState& s = e->st;
  return e->d_gid && e->d_rev && s.E[0] && s.E[1] && s.E[0] != s.E[1] && s.AW[0] &&
         e->W > GROUPED_W_MAX && e->W <= 64;
}

// Run this round's update and its (dense) pushes in one pass?
bool update_push_round(const p2pg_engine* e, const RoundParams& p) {
  if (e->update_push == 0 || e->cfg.mode != P2PG_MODE_GOSSIP || e->push_mode != 0 || e->d_gid ||
      p.phase >= 0 || !e->st.E[0] || !wide_atomic_on(e) || !gossip_update_push_supported(e->st))
    return false;
  return e->update_push == 1 || predict_dense(e);
}

// After the stream synced on a round whose push ran lane-parallel: the list must have held
// every (peer, word) pair (n_words is the frontier's own count, so a shortfall is a bug).
int check_scatter_list(p2pg_engine* e, unsigned long long listed) {
  if (!e->wlist_check) return P2PG_OK;
  e->wlist_check = false;
  if ((int64_t)listed > e->wlist_cap)
    return fail(e, P2PG_ERR_STATE, "sparse scatter: " + std::to_string(listed) +
                                          " frontier words listed, room for " +
                                          std::to_string(e->wlist_cap));
  return P2PG_OK;
}

// Arrivals (p2pg_round_stats.received): a churn run with P2PG_FLAG_RECEIVED counts the lost sends
// of every round.
bool count_lost_on(const p2pg_engine* e) {
  return e->cfg.churn_threshold != 0 && (e->cfg.flags & P2PG_FLAG_RECEIVED);
}
// Is the `received` counter exact (no churn, or churn losses counted)?
bool received_exact(const p2pg_engine* e) { return e->cfg.churn_threshold == 0 || count_lost_on(e); }

// Enqueue the count of round r's lost sends (k_sends, count mode) over gs (the graph the sends
// leave on; gone slots = removed connections) and gp (the graph round r's arrivals travelled
// on: the senders' own first receipts); the count lands in h_cnt2[1] at the next stream sync.
hipError_t enqueue_lost_count(p2pg_engine* e, const DevGraph& gs, const DevGraph& gp, int32_t r) {
  hipError_t x = hipMemsetAsync(e->d_cnt2, 0, 2 * sizeof(unsigned long long), e->stream);
  RoundParams p = params(e);
  p.round = r;
  if (x == hipSuccess)
    x = launch_sends(gs, gp, e->st, p, false, 0, nullptr, nullptr, nullptr, nullptr, e->d_cnt2, e->stream);
  if (x == hipSuccess)
    x = hipMemcpyAsync(e->h_cnt2, e->d_cnt2, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->stream);
  return x;
}

// Dense-round edge-mask planes E, sized by the current nnz: one, or two for fused rounds
// (round r pulls E[(r-1)&1], pushes E[r&1]); only if they fit with headroom -- else gossip
// pushes by row atomics only.  Replaces any previous planes (their contents are dropped).
int alloc_edge_planes(p2pg_engine* e) {
  DevState& s = e->st;
  if (s.E[1] == s.E[0]) s.E[1] = nullptr;
  dfree(s.E[0]);
  dfree(s.E[1]);
  if (e->cfg.mode != P2PG_MODE_GOSSIP || !e->d_rev || e->push_mode == 1) return P2PG_OK;
  // a rank-local graph's ghost slots are usable by the PART kernels only (part_dense)
  if ((e->cfg.flags & P2PG_FLAG_LOCAL_GRAPH) &&
      !(e->fused && e->W > GROUPED_W_MAX && e->W <= 64 && s.AW[0]))
    return P2PG_OK;
  const size_t eb = (size_t)e->nnz * e->W * sizeof(uint64_t);
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || eb + ((size_t)4 << 30) >= free_b)
    return P2PG_OK;
  HIPCHK(e, hipMalloc((void**)&s.E[0], eb ? eb : 8));
  s.E[1] = s.E[0];
  if (e->W <= 64 && e->fused && hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
      eb + ((size_t)4 << 30) < free_b)
    HIPCHK(e, hipMalloc((void**)&s.E[1], eb ? eb : 8));
  return P2PG_OK;
}

int alloc_state(p2pg_engine* e) {
  free_state(e);
  DevState& s = e->st;
  s.W = e->W;
  e->e_thresh = e->e_thresh_env >= 0.0 ? e->e_thresh_env : (e->W > GROUPED_W_MAX ? 0.06 : 0.04);
  // a dense round costs a visit of every unsaturated peer whatever the width, a sparse one an
  // atomic per pushed mask: narrow rows (a message split's shares) stay sparse until nearly every
  // peer is active (c4 interleaved sweeps, profiles/r03/ab_v_thresh.txt: W = 8 0.3 / 0.6 / 0.9 /
  // 0.95 / 0.98 -> 85.6 / 81.3 / 79.9 / 79.2 / 83.6 ms; W = 16 -> 144.5 / 138.9 / 130.4 / 128.7 /
  // 127.6 ms; W = 32 0.3 / 0.7 / 0.9 / 0.95 -> 218.4 / 211.7 / 208.4 / 203.7 ms; W = 64: 0.3 ...
  // 0.9 equal, 0.95 within 1 %, so the round-2 value stays)
  e->v_thresh = e->v_thresh_env >= 0.0 ? e->v_thresh_env : e->W <= 32 ? 0.95 : 0.3;
  s.M = e->M;
  e->plane_bytes = (size_t)e->V * e->W * sizeof(uint64_t);
  e->seen_spare_off = false;  // a new plane size: the spare's size / memory check runs again
  e->bm_bytes = (size_t)((e->V + 31) / 32) * sizeof(uint32_t);
  const bool gossip = e->cfg.mode == P2PG_MODE_GOSSIP;
  const bool rec = (e->cfg.flags & P2PG_FLAG_RECORD) != 0;
  auto A = [&](void** p, size_t n) -> int {
    hipError_t r = hipMalloc(p, n ? n : 8);
    if (r != hipSuccess) {
      free_state(e);
      return fail(e, r == hipErrorOutOfMemory ? P2PG_ERR_NOMEM : P2PG_ERR_HIP,
                  std::string("hipMalloc: ") + hipGetErrorString(r));
    }
    return P2PG_OK;
  };
  int rc;
  if ((rc = A((void**)&s.seen, e->plane_bytes))) return rc;
  for (int i = 0; i < 2; ++i) {
    if ((rc = A((void**)&s.F[i], e->plane_bytes))) return rc;
    if ((rc = A((void**)&s.A[i], e->bm_bytes))) return rc;
    if (gossip) {
      if ((rc = A((void**)&s.next[i], e->plane_bytes))) return rc;
      if ((rc = A((void**)&s.T[i], e->bm_bytes))) return rc;
      HIPCHK(e, hipMemsetAsync(s.next[i], 0, e->plane_bytes, e->stream));
      HIPCHK(e, hipMemsetAsync(s.T[i], 0, e->bm_bytes, e->stream));
    }
  }
  if ((rc = A((void**)&s.S, e->bm_bytes))) return rc;
  if (gossip && e->W > PACK_W_MAX_PLAIN && e->W <= 64)  // packed E rows (see DevState::AW)
    for (int i = 0; i < 2; ++i)
      if ((rc = A((void**)&s.AW[i], sizeof(uint64_t) * (size_t)e->V))) return rc;
  if ((rc = alloc_edge_planes(e))) {
    free_state(e);
    return rc;
  }
  if (rec) {
    const size_t hb = (size_t)e->V * e->M * sizeof(int32_t);
    if ((rc = A((void**)&s.hop, hb))) return rc;
    if ((rc = A((void**)&s.parent, hb))) return rc;
  }
  if ((rc = A((void**)&s.stats, STAT_BYTES))) return rc;
  if ((rc = A((void**)&e->d_cnt2, 2 * sizeof(unsigned long long)))) return rc;
  HIPCHK(e, hipHostMalloc((void**)&e->h_cnt2, 2 * sizeof(unsigned long long)));
#ifdef P2PG_PROF
  if ((rc = A((void**)&s.prof, sizeof(unsigned long long) * 16))) return rc;
  HIPCHK(e, hipMemset(s.prof, 0, sizeof(unsigned long long) * 16));
#endif
  if ((rc = A((void**)&e->d_src, sizeof(int32_t) * (e->M ? e->M : 1)))) return rc;
  e->have_state = true;
  e->stats_clear = true;
  return P2PG_OK;
}

}  // namespace

extern "C" {

int p2pg_create(const p2pg_config* cfg, p2pg_engine** out) {
  if (!cfg || !out) return fail(nullptr, P2PG_ERR_ARG, "create: null argument");
  *out = nullptr;
  if (cfg->mode != P2PG_MODE_FLOOD && cfg->mode != P2PG_MODE_GOSSIP)
    return fail(nullptr, P2PG_ERR_ARG, "create: unknown mode");
  if (cfg->mode == P2PG_MODE_GOSSIP && (cfg->fanout < 1 || cfg->fanout > 16))
    return fail(nullptr, P2PG_ERR_ARG, "create: gossip fanout must be in [1, 16]");
  int ndev = 0;
  hipError_t r = hipGetDeviceCount(&ndev);
  if (r != hipSuccess || ndev == 0)
    return fail(nullptr, P2PG_ERR_HIP, "create: no HIP device visible");
  if (cfg->device < 0 || cfg->device >= ndev)
    return fail(nullptr, P2PG_ERR_ARG, "create: device ordinal out of range");
  p2pg_engine* e = new p2pg_engine;
  e->cfg = *cfg;
  if (const char* t = std::getenv("P2PG_E_THRESH")) e->e_thresh_env = std::atof(t);
  if (const char* t = std::getenv("P2PG_V_THRESH")) e->v_thresh_env = std::atof(t);
  if (const char* f = std::getenv("P2PG_FUSED")) e->fused = std::strcmp(f, "0") != 0;
  if (const char* f = std::getenv("P2PG_SPARSE_LP")) e->sparse_lp = std::strcmp(f, "0") != 0;
  if (const char* f = std::getenv("P2PG_PUSH_DEDUP")) e->push_dedup = std::atoi(f);
  if (const char* f = std::getenv("P2PG_WIDE_ATOMIC")) e->wide_atomic = std::strcmp(f, "0") != 0;
  if (const char* f = std::getenv("P2PG_UPDATE_PUSH")) e->update_push = std::atoi(f);
  if (const char* f = std::getenv("P2PG_RUN_BATCH")) e->batch_rounds = std::atoi(f);
  if (const char* f = std::getenv("P2PG_DECAY_PRED")) e->decay_pred = std::strcmp(f, "0") != 0;
  if (const char* f = std::getenv("P2PG_PARTIAL_F")) e->partial_f = std::strcmp(f, "0") != 0;
  if (const char* f = std::getenv("P2PG_SEEN_SPARE")) e->seen_spare_on = std::strcmp(f, "0") != 0;
  if (const char* m = std::getenv("P2PG_GOSSIP_PUSH"))
    e->push_mode = !std::strcmp(m, "atomic") ? 1 : (!std::strcmp(m, "store") ? 2 : 0);
  HIPCHK(e, hipSetDevice(cfg->device));
  HIPCHK(e, hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking));
  e->stream = e->own_stream;
  HIPCHK(e, hipEventCreate(&e->ev[0]));
  HIPCHK(e, hipEventCreate(&e->ev[1]));
  HIPCHK(e, hipEventCreateWithFlags(&e->ev_sync, hipEventDisableTiming));
  if (const char* f = std::getenv("P2PG_SPIN")) e->spin = std::strcmp(f, "0") != 0;
  HIPCHK(e, hipHostMalloc((void**)&e->h_stats, STAT_BYTES));
  *out = e;
  return P2PG_OK;
}

int p2pg_set_stream(p2pg_engine* e, void* hip_stream) {
  if (!e) return P2PG_ERR_ARG;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : e->own_stream;
  if (s != e->stream && e->stream) {  // work queued on the old stream finishes first
    HIPCHK(e, hipSetDevice(e->cfg.device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  e->stream = s;
  return P2PG_OK;
}

}  // extern "C"

namespace {

// Checks the CSR invariants the kernels rely on and builds the gossip reverse slots.
int check_csr(p2pg_engine* e, int64_t V, const int64_t* rowptr, const int32_t* colidx,
              std::vector<uint32_t>& rev) {
  if (V <= 0 || V > 0x7FFFFFFFll || !rowptr) return fail(e, P2PG_ERR_ARG, "load_csr: bad arguments");
  const int64_t nnz = rowptr[V];
  if (rowptr[0] != 0 || nnz < 0 || (nnz > 0 && !colidx))
    return fail(e, P2PG_ERR_GRAPH, "load_csr: rowptr[0] must be 0 and rowptr[V] >= 0");
  // validate: monotone rows, ids in range, strictly ascending (sorted, no multi-edges),
  // no self loops -- the invariants the kernels' lowest-id parent order relies on
  for (int64_t v = 0; v < V; ++v) {
    if (rowptr[v + 1] < rowptr[v]) return fail(e, P2PG_ERR_GRAPH, "load_csr: rowptr not monotone");
    for (int64_t j = rowptr[v]; j < rowptr[v + 1]; ++j) {
      const int32_t u = colidx[j];
      if (u < 0 || u >= V) return fail(e, P2PG_ERR_GRAPH, "load_csr: neighbour id out of range");
      if (u == v) return fail(e, P2PG_ERR_GRAPH, "load_csr: self loop");
      if (j > rowptr[v] && colidx[j - 1] >= u)
        return fail(e, P2PG_ERR_GRAPH, "load_csr: row not strictly ascending");
    }
  }
  // symmetry (every connection relays both ways, node.py:75-78) and reverse slots
  const bool local = (e->cfg.flags & P2PG_FLAG_LOCAL_GRAPH) != 0;
  // reverse slots for gossip's dense rounds; on a rank-local graph a ghost neighbour's slot is
  // marked instead (REV_GHOST | its local id), and slot ids must stay below that bit
  rev.assign(e->cfg.mode == P2PG_MODE_GOSSIP && nnz < (local ? (int64_t)REV_GHOST : 0xFFFFFFFFll) ? nnz : 0,
             0u);
  int64_t asym = -1;
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t u = 0; u < V; ++u) {
    for (int64_t j = rowptr[u]; j < rowptr[u + 1]; ++j) {
      const int64_t v = colidx[j];
      const int32_t* b = colidx + rowptr[v];
      const int32_t* en = colidx + rowptr[v + 1];
      if (local && b == en) {  // ghost peer: its row lives on its owner rank
        if (!rev.empty()) rev[j] = REV_GHOST | (uint32_t)v;
        continue;
      }
      const int32_t* it = std::lower_bound(b, en, (int32_t)u);
      if (it == en || *it != u) {
#pragma omp critical
        asym = u;
      } else if (!rev.empty()) {
        rev[j] = (uint32_t)(rowptr[v] + (it - b));
      }
    }
  }
  if (asym >= 0) return fail(e, P2PG_ERR_GRAPH, "load_csr: adjacency not symmetric");
  return P2PG_OK;
}

// Device copies of a checked CSR (rows, reverse slots, gossip chunk items, pull hub plan);
// replaces the engine's topology arrays, leaves the run state alone.
int upload_graph(p2pg_engine* e, int64_t V, const int64_t* rowptr, const int32_t* colidx,
                 const std::vector<uint32_t>& rev) {
  const int64_t nnz = rowptr[V];
  free_topology(e);
  e->V = V;
  e->nnz = nnz;
  e->v_conn = 0;
  for (int64_t v = 0; v < V; ++v) e->v_conn += rowptr[v + 1] > rowptr[v];
  if (!rev.empty()) {
    HIPCHK(e, hipMalloc((void**)&e->d_rev, sizeof(uint32_t) * rev.size()));
    HIPCHK(e, hipMemcpy(e->d_rev, rev.data(), sizeof(uint32_t) * rev.size(), hipMemcpyHostToDevice));
  }
  e->h_rowptr.assign(rowptr, rowptr + V + 1);
  e->seed.ok = false;
  e->h_colidx.assign(colidx, colidx + nnz);
  HIPCHK(e, hipMalloc((void**)&e->d_rowptr, sizeof(int64_t) * (V + 1)));
  HIPCHK(e, hipMalloc((void**)&e->d_colidx, sizeof(int32_t) * (nnz ? nnz : 1)));
  HIPCHK(e, hipMemcpy(e->d_rowptr, rowptr, sizeof(int64_t) * (V + 1), hipMemcpyHostToDevice));
  if (nnz) HIPCHK(e, hipMemcpy(e->d_colidx, colidx, sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
  // gossip: (source, neighbour-chunk) items for sources wider than one chunk
  std::vector<int64_t> hub, hub_big;
  std::vector<int32_t> wide_big;
  for (int64_t v = 0; v < V; ++v) {
    const int64_t d = rowptr[v + 1] - rowptr[v];
    if (d > GCHUNK) {
      if (d > HUB_T) wide_big.push_back((int32_t)v);
      for (int64_t c = 0; c * GCHUNK < d; ++c) {
        hub.push_back((v << 32) | c);
        if (d > HUB_T) hub_big.push_back((v << 32) | c);
      }
    }
  }
  e->n_wide_big = (int64_t)wide_big.size();
  if (!wide_big.empty()) {
    HIPCHK(e, hipMalloc((void**)&e->d_wide_big, sizeof(int32_t) * wide_big.size()));
    HIPCHK(e, hipMemcpy(e->d_wide_big, wide_big.data(), sizeof(int32_t) * wide_big.size(), hipMemcpyHostToDevice));
  }
  e->n_hub = (int64_t)hub.size();
  e->n_hub_big = (int64_t)hub_big.size();
  {  // pull-side hub plan
    std::vector<int32_t> hubs;
    std::vector<int64_t> items, begin{0};
    std::vector<uint32_t> H((V + 31) / 32, 0u);
    for (int64_t v = 0; v < V; ++v) {
      const int64_t d = rowptr[v + 1] - rowptr[v];
      if (d <= HUB_T) continue;
      hubs.push_back((int32_t)v);
      H[v >> 5] |= 1u << (v & 31);
      for (int64_t c = 0; c * HUB_CHUNK < d; ++c) items.push_back((v << 32) | c);
      begin.push_back((int64_t)items.size());
    }
    HIPCHK(e, hipMalloc((void**)&e->d_H, sizeof(uint32_t) * H.size()));
    HIPCHK(e, hipMemcpy(e->d_H, H.data(), sizeof(uint32_t) * H.size(), hipMemcpyHostToDevice));
    if (!hubs.empty()) {
      HIPCHK(e, hipMalloc((void**)&e->d_hubs, sizeof(int32_t) * hubs.size()));
      HIPCHK(e, hipMalloc((void**)&e->d_hub_items, sizeof(int64_t) * items.size()));
      HIPCHK(e, hipMalloc((void**)&e->d_hub_begin, sizeof(int64_t) * begin.size()));
      HIPCHK(e, hipMalloc((void**)&e->d_partial, sizeof(uint64_t) * 64 * items.size()));
      HIPCHK(e, hipMemcpy(e->d_hubs, hubs.data(), sizeof(int32_t) * hubs.size(), hipMemcpyHostToDevice));
      HIPCHK(e, hipMemcpy(e->d_hub_items, items.data(), sizeof(int64_t) * items.size(), hipMemcpyHostToDevice));
      HIPCHK(e, hipMemcpy(e->d_hub_begin, begin.data(), sizeof(int64_t) * begin.size(), hipMemcpyHostToDevice));
    }
    e->hp = HubPlan{e->d_hub_items, (int64_t)items.size(), e->d_hubs, e->d_hub_begin,
                    (int64_t)hubs.size(), e->d_partial};
    // the fused kernels' push modes skip the H peers and push them through wide_big
    // (launch_wide_push_e): the two sets must be the same peers
    if (hubs.size() != wide_big.size() || !std::equal(hubs.begin(), hubs.end(), wide_big.begin()))
      return fail(e, P2PG_ERR_STATE, "load_csr: pull hubs and wide push sources differ");
  }
  HIPCHK(e, hipMalloc((void**)&e->d_hub, sizeof(int64_t) * (hub.empty() ? 1 : hub.size())));
  if (!hub.empty())
    HIPCHK(e, hipMemcpy(e->d_hub, hub.data(), sizeof(int64_t) * hub.size(), hipMemcpyHostToDevice));
  HIPCHK(e, hipMalloc((void**)&e->d_hub_big, sizeof(int64_t) * (hub_big.empty() ? 1 : hub_big.size())));
  if (!hub_big.empty())
    HIPCHK(e, hipMemcpy(e->d_hub_big, hub_big.data(), sizeof(int64_t) * hub_big.size(), hipMemcpyHostToDevice));
  return P2PG_OK;
}

}  // namespace

extern "C" {

int p2pg_load_csr(p2pg_engine* e, int64_t V, const int64_t* rowptr, const int32_t* colidx) {
  if (!e) return fail(e, P2PG_ERR_ARG, "load_csr: bad arguments");
  std::vector<uint32_t> rev;
  int rc = check_csr(e, V, rowptr, colidx, rev);
  if (rc) return rc;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  free_graph(e);
  free_state(e);
  if ((rc = upload_graph(e, V, rowptr, colidx, rev))) return rc;
  e->M = 0;
  e->W = 0;
  e->round = 0;
  e->done = true;
  return P2PG_OK;
}

int p2pg_set_sources(p2pg_engine* e, int32_t M, const int32_t* src) {
  if (!e || M <= 0 || !src) return fail(e, P2PG_ERR_ARG, "set_sources: need M > 0 and src");
  if (!e->d_rowptr) return fail(e, P2PG_ERR_STATE, "set_sources: load a graph first");
  for (int32_t m = 0; m < M; ++m)
    if (src[m] < 0 || src[m] >= e->V) return fail(e, P2PG_ERR_ARG, "set_sources: source out of range");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  const int32_t W = (M + 63) / 64;
  e->h_src.assign(src, src + M);
  e->seed.ok = false;
  if (!e->have_state || W != e->W || M != e->M) {
    e->M = M;
    e->W = W;
    int rc = alloc_state(e);
    if (rc) return rc;
  }
  HIPCHK(e, hipMemcpy(e->d_src, src, sizeof(int32_t) * M, hipMemcpyHostToDevice));
  return p2pg_reset(e);
}

}  // extern "C"

namespace {

// Round 0's counters: the originations, from the host copies of the sources and the rows (the
// seed kernel counts nothing).  They depend on the sources and the graph only, so they are
// computed once per p2pg_set_sources / p2pg_load_csr rather than per run: a run's round 0 used to
// sort the sources on the host while the GPU waited (~0.25 ms per c4 step).
const SeedStats& seed_stats(p2pg_engine* e) {
  SeedStats& ss = e->seed;
  if (ss.ok) return ss;
  ss = SeedStats{};
  const bool gossip = e->cfg.mode == P2PG_MODE_GOSSIP;
  std::vector<int64_t> vs(e->h_src.begin(), e->h_src.end());
  std::vector<int64_t> vw(e->M);
  for (int32_t m = 0; m < e->M; ++m) {
    const int64_t v = e->h_src[m];
    const int64_t d = e->h_rowptr[v + 1] - e->h_rowptr[v];
    ss.relays += gossip ? (uint64_t)std::min<int64_t>(d, e->cfg.fanout) : (uint64_t)d;
    vw[m] = v * e->W + (m >> 6);
  }
  ss.nw = (uint64_t)e->M;
  std::sort(vs.begin(), vs.end());
  vs.erase(std::unique(vs.begin(), vs.end()), vs.end());
  std::sort(vw.begin(), vw.end());
  vw.erase(std::unique(vw.begin(), vw.end()), vw.end());
  ss.av = vs.size();
  ss.aw = vw.size();
  for (int64_t v : vs) ss.degact += (uint64_t)(e->h_rowptr[v + 1] - e->h_rowptr[v]);
  for (int64_t x : vw) {
    const int64_t v = x / e->W;
    ss.wedge += (uint64_t)(e->h_rowptr[v + 1] - e->h_rowptr[v]);
  }
  ss.ok = true;
  return ss;
}

// p2pg_reset's spare seen plane (p2pg_engine::seen_spare): allocated on first use; false when
// disabled or when the device has no room for it (then it stays disabled)
bool spare_ready(p2pg_engine* e) {
  if (!e->seen_spare_on || e->seen_spare_off) return false;
  if (e->seen_spare) return true;
  // only where it is cheap: a plane of at most 1/16 of the device (config 4: 5.1 GB of 288) with
  // room to spare, so that the copy never takes the memory a larger run (config 5's 51 GB planes,
  // several engines of one process) needs
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || e->plane_bytes > total_b / 16 ||
      free_b < 4 * e->plane_bytes) {
    (void)hipGetLastError();
    e->seen_spare_off = true;
    return false;
  }
  if (!e->side) {
    if (hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_spare, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_main, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      e->seen_spare_off = true;
      return false;
    }
  }
  if (hipMalloc((void**)&e->seen_spare, e->plane_bytes) != hipSuccess) {
    (void)hipGetLastError();
    e->seen_spare = nullptr;
    e->seen_spare_off = true;
    return false;
  }
  e->spare_pending = false;
  return true;
}

}  // namespace

extern "C" {

int p2pg_reset(p2pg_engine* e) {
  if (!e || !e->have_state) return fail(e, P2PG_ERR_STATE, "reset: no sources set");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  DevState& s = e->st;
  if (!spare_ready(e)) {
    HIPCHK(e, hipMemsetAsync(s.seen, 0, e->plane_bytes, e->stream));
  } else {
    if (e->spare_pending) {  // the spare is zero once the side stream's zeroing has run
      HIPCHK(e, hipStreamWaitEvent(e->stream, e->ev_spare, 0));
      std::swap(s.seen, e->seen_spare);
    } else {  // (first reset with a spare: zero the plane in use here, the spare below)
      HIPCHK(e, hipMemsetAsync(s.seen, 0, e->plane_bytes, e->stream));
    }
    // the replaced plane: zeroed on the side stream after everything queued so far has read it
    HIPCHK(e, hipEventRecord(e->ev_main, e->stream));
    HIPCHK(e, hipStreamWaitEvent(e->side, e->ev_main, 0));
    HIPCHK(e, hipMemsetAsync(e->seen_spare, 0, e->plane_bytes, e->side));
    HIPCHK(e, hipEventRecord(e->ev_spare, e->side));
    e->spare_pending = true;
  }
  HIPCHK(e, hipMemsetAsync(s.S, 0, e->bm_bytes, e->stream));
  for (int i = 0; i < 2; ++i) HIPCHK(e, hipMemsetAsync(s.A[i], 0, e->bm_bytes, e->stream));
  if (s.next[0] && ((!e->done && e->round > 0) || e->consume_next)) {
    // an interrupted run may leave pushes / materialized arrivals in flight: clear them
    for (int i = 0; i < 2; ++i) {
      HIPCHK(e, hipMemsetAsync(s.next[i], 0, e->plane_bytes, e->stream));
      HIPCHK(e, hipMemsetAsync(s.T[i], 0, e->bm_bytes, e->stream));
    }
  }
  if (s.hop) {
    HIPCHK(e, hipMemsetAsync(s.hop, 0xFF, (size_t)e->V * e->M * sizeof(int32_t), e->stream));
    HIPCHK(e, hipMemsetAsync(s.parent, 0xFF, (size_t)e->V * e->M * sizeof(int32_t), e->stream));
  }
  e->round = 0;
  e->done = false;
  e->failed.clear();
  e->stats_clear = true;
  e->begun = false;
  e->auto_round = -1;
  e->frontier_kept = true;
  e->frontier_kept_prev = true;
  e->last_push_e = false;
  e->consume_next = false;
  e->total_relays = 0;
  e->sent_last = e->lost_last = 0;
  free_arr(e);
  e->prev_aw = e->prev_av = 0;
  e->last_new = 0;
  e->prev2_aw = e->prev2_av = e->prev2_new = 0;
  e->prev_sw = 0;
  e->saw_dense = false;
  // (a previous run's unresolved launch timings belong to it, not to the next one)
  e->ev_cls.clear();
  for (int i = 0; i < P2PG_KCLASS_N; ++i) {
    e->kms[i] = 0;
    e->klaunch[i] = 0;
  }
  return P2PG_OK;
}

}  // extern "C"

namespace {

// Can this round's pull / update run in two phases (interior peers, then border peers)?
// Vertex-partitioned ranks with ghosts, rounds r >= 1 of the flood pull or the gossip update.
bool split_round(const p2pg_engine* e) {
  return e->d_border && e->round > 0 && !e->consume_next &&
         (e->cfg.mode == P2PG_MODE_FLOOD || !e->last_push_e);
}

}  // namespace

extern "C" {

int p2pg_step_begin(p2pg_engine* e) {
  if (!e || !e->have_state) return fail(e, P2PG_ERR_STATE, "step_begin: no sources set");
  if (!e->failed.empty()) return fail(e, P2PG_ERR_STATE, "step_begin: " + e->failed);
  if (e->begun) return fail(e, P2PG_ERR_STATE, "step_begin: the round has begun already");
  // a rank-local graph marks its ghost slots REV_GHOST | id, which only the PART kernels (global
  // ids set) know: the one-GPU kernels would index E with them
  if ((e->cfg.flags & P2PG_FLAG_LOCAL_GRAPH) && !e->d_gid)
    return fail(e, P2PG_ERR_STATE, "step_begin: a local-graph engine needs p2pg_set_global_ids first");
  if (e->done) return P2PG_OK;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  DevState& s = e->st;
  if (e->stats_clear) {
    HIPCHK(e, hipMemsetAsync(s.stats, 0, STAT_BYTES, e->stream));
    std::memset(e->stats_base, 0, sizeof(e->stats_base));
    e->stats_clear = false;
  }
  e->begun = true;
  if (!split_round(e)) return P2PG_OK;
  // phase 0: peers without a ghost neighbour, which need none of the rows still in transit
  const DevGraph g = graph(e);
  RoundParams p = params(e);
  p.border = e->d_border;
  p.phase = 0;
  if (e->cfg.mode == P2PG_MODE_FLOOD)
    return timed(e, 1, [&] { return launch_flood_pull(g, s, p, e->hp, e->stream); });
  return timed(e, 4, [&] { return launch_gossip_update(g, s, p, e->stream); });
}

int p2pg_step(p2pg_engine* e, p2pg_round_stats* out) {
  if (!e || !e->have_state) return fail(e, P2PG_ERR_STATE, "step: no sources set");
  if (!e->failed.empty()) return fail(e, P2PG_ERR_STATE, "step: " + e->failed);
  if (e->done) {
    e->begun = false;
    if (out) {
      std::memset(out, 0, sizeof(*out));
      out->round = e->round;
    }
    return 0;
  }
  int rc;
  if (!e->begun && (rc = p2pg_step_begin(e))) return rc;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  DevState& s = e->st;
  if (e->arr_round >= 0 && e->round > e->arr_round) free_arr(e);
  const DevGraph g = graph(e);
  RoundParams p = params(e);
  if (split_round(e)) {  // phase 0 ran in step_begin: the border peers now
    p.border = e->d_border;
    p.phase = 1;
  }
  e->begun = false;
  const bool gossip = e->cfg.mode == P2PG_MODE_GOSSIP;
  bool fused_round = false, up_round = false;
  // the update / pull-only pass of this round (fused and update+push rounds set their own)
  if (gossip && partial_frontier(e, e->skip_frontier)) p.store_f = 2;
  uint64_t host_new = 0, host_relays = 0, host_av = 0, host_aw = 0, host_wedge = 0, host_degact = 0;
  if (e->round == 0) {
    if ((rc = timed(e, 0, [&] { return launch_zero_rows(s.F[0], e->W, e->d_src, e->M, e->stream); }))) return rc;
    if (s.AW[0])
      if ((rc = timed(e, 0, [&] { return launch_zero_rows(s.AW[0], 1, e->d_src, e->M, e->stream); }))) return rc;
    if ((rc = timed(e, 0, [&] { return launch_seed(s, e->d_src, e->M, e->stream); }))) return rc;
    // origination stats from the host copy of the sources (computed once per sources and graph)
    const SeedStats& ss = seed_stats(e);
    host_new = ss.nw;
    host_relays = ss.relays;
    host_av = ss.av;
    host_aw = ss.aw;
    host_wedge = ss.wedge;
    host_degact = ss.degact;
  } else if (e->consume_next) {
    // arrivals materialized into row pushes (topology update / restored snapshot)
    if ((rc = timed(e, 4, [&] { return launch_gossip_update(g, s, p, e->stream); }))) return rc;
    e->consume_next = false;
  } else if (!gossip) {
    if ((rc = timed(e, 1, [&] { return launch_flood_pull(g, s, p, e->hp, e->stream); }))) return rc;
  } else if (e->last_push_e) {
    // previous round stored per-edge masks: gather them (pull, no atomics).  If this round is
    // predicted dense as well (the previous round's word density; the prediction only picks
    // the push form, never the result), the same pass also pushes this round's receipts.
    const bool dense_pred = e->push_mode == 2 || (e->push_mode == 0 && still_dense(e));
    const bool part = e->d_gid != nullptr;  // (a rank gets here only if part_dense)
    fused_round = (!part || part_dense(e)) && dense_pred && gossip_fused_supported(s);
    if (fused_round) {
      // a frontier nobody observes is not stored: inside p2pg_run (not its last allowed
      // round), without hop/parent records
      p.store_f = (e->skip_frontier && !s.hop) ? 0 : 1;
      if ((rc = timed(e, 7, [&] { return launch_fused_round(e, g, p); }))) return rc;
    } else {
      if ((rc = timed(e, 5, [&] {
             hipError_t r = launch_gossip_pull(g, s, p, e->hp, e->stream);
             return r != hipSuccess || !part ? r : launch_clear_arrivals(s, p.round, e->V, e->stream);
           })))
        return rc;
    }
  } else if (update_push_round(e, p)) {
    // the first dense round after a sparse one: update and E pushes in one pass (timed with the
    // store pushes); the frontier rows follow the fused rounds' rule
    up_round = true;
    p.store_f = (e->skip_frontier && !s.hop) ? 0 : 1;
    if ((rc = timed(e, 6, [&] {
           return launch_gossip_update_push(g, s, p, e->d_hub_big, e->n_hub_big, e->d_wide_big,
                                            e->n_wide_big, e->stream);
         })))
      return rc;
  } else {
    if ((rc = timed(e, 4, [&] { return launch_gossip_update(g, s, p, e->stream); }))) return rc;
  }
  if (s.hop)
    if ((rc = timed(e, 3, [&] {
           return launch_record(graph_for_arrivals(e, e->round), s, p, e->stream);
         })))
      return rc;
  uint64_t tot[STAT_N] = {0};
  auto read_stats = [&]() -> int {
    HIPCHK(e, hipMemcpyAsync(e->h_stats, s.stats, STAT_BYTES, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, round_sync(e));
    int r2 = resolve_timings(e);
    if (r2) return r2;
    for (int i = 0; i < STAT_N; ++i) tot[i] = 0;
    for (int sh = 0; sh < STAT_SHARDS; ++sh)
      for (int i = 0; i < STAT_N; ++i)
        tot[i] += e->h_stats[sh * STAT_N + i] - e->stats_base[sh * STAT_N + i];
    if (e->round == 0) {
      tot[ST_NEW] = host_new;
      tot[ST_RELAYS] = host_relays;
      tot[ST_ACTIVE_V] = host_av;
      tot[ST_ACTIVE_W] = host_aw;
      tot[ST_WEDGES] = host_wedge;
      tot[ST_DEG_ACT] = host_degact;
    }
    return P2PG_OK;
  };
  if (gossip && (fused_round || up_round)) {
    e->last_push_e = true;  // the fused launches pushed every source of this round
  } else if (gossip) {
    // push form for this round's sends: row atomics when the frontier is sparse, whole-row
    // edge-mask stores (+ pull next round) when most words of the active rows are set
    bool use_e = false, have_tot = false;
    // the counters of this round are needed before its push only to choose the form (unless
    // that choice is clear already) and to size the sparse push's (peer, word) list (else
    // bounded by the last round's pushed masks).  Not on a vertex-partitioned rank: rows other
    // ranks pushed arrive by the exchange, so this rank's own pushed masks bound nothing
    const bool blind = e->round > 0 && e->push_mode != 2 && !e->d_gid && clearly_sparse(e) &&
                       e->prev_sw > 0;
    // (partitioned ranks: E for their local connections when part_dense, ghost rows travel)
    if (s.E[0] && (!e->d_gid || part_dense(e))) {
      if (e->push_mode == 2) {
        use_e = true;
      } else if (e->push_mode == 0 && !blind) {
        if (e->round == 0) {  // round 0's counters are the host's (seed_stats): no read-back
          tot[ST_ACTIVE_W] = host_aw;
          tot[ST_ACTIVE_V] = host_av;
        } else if ((rc = read_stats())) {
          return rc;
        }
        have_tot = true;
        use_e = (double)tot[ST_ACTIVE_W] >=
                e->e_thresh * (double)tot[ST_ACTIVE_V] * (double)e->W && tot[ST_ACTIVE_V] > 0 &&
                (double)tot[ST_ACTIVE_V] >= e->v_thresh * (double)e->v_conn;
      }
    }
    // the lane-parallel sparse push sizes its (peer, word) list by the frontier's word count
    if (!use_e && !have_tot && !blind && sparse_scatter_on(e)) {
      if (e->round == 0) {
        tot[ST_ACTIVE_W] = host_aw;
        tot[ST_ACTIVE_V] = host_av;
      } else if ((rc = read_stats())) {
        return rc;
      }
      have_tot = true;
    }
    // decay phase (fewer first receipts than the round before): most pushes are duplicates,
    // so the sparse push drops seen bits before its atomics (RoundParams::dedup_push).  The
    // phase is "after the dense rounds" (saw_dense), a fact every schedule agrees on -- a
    // batched decay round, a blind push and a round that read its counters first must filter
    // alike, because the filter decides which fully-seen masks are still pushed, i.e. the
    // touched-words counter of the next round (results never depend on it)
    if (!use_e && sparse_scatter_on(e))
      p.dedup_push = e->push_dedup == 1 || (e->push_dedup < 0 && e->saw_dense);
    const uint64_t list_words = have_tot ? tot[ST_ACTIVE_W] : e->prev_sw;
    if ((rc = timed(e, use_e ? 6 : 2, [&] {
           return use_e ? launch_gossip_scatter(g, s, p, e->d_hub, e->n_hub, true, e->stream,
                                                e->d_hub_big, e->n_hub_big, e->d_wide_big,
                                                e->n_wide_big)
                        : launch_scatter_atomic(e, g, p, list_words);
         })))
      return rc;
    e->last_push_e = use_e;
  }
  if (e->auto_buf && e->d_seg_cnt) {
    // partitioned ranks: pack this round's live boundary rows now, so the one synchronisation
    // below (the round counters) also covers the pack and its counts -- no second drain of the
    // stream before the records leave (p2pg_set_exchange_buffer)
    const bool fwd = e->auto_plane == 0;
    const int nseg = (int)e->send_seg.size() - 1;
    HIPCHK(e, hipMemsetAsync(e->d_seg_cnt, 0, sizeof(unsigned long long) * P2PG_MAX_RANKS, e->stream));
    hipError_t r = launch_pack_live(s, e->auto_plane, e->round, fwd ? e->d_send : e->d_recv,
                                    fwd ? e->n_send : e->n_recv, fwd ? e->d_send_seg : e->d_recv_seg,
                                    nseg, e->d_seg_cnt, (int64_t*)e->auto_buf, e->stream);
    if (r == hipSuccess)
      r = hipMemcpyAsync(e->h_seg_cnt, e->d_seg_cnt, sizeof(unsigned long long) * nseg,
                         hipMemcpyDeviceToHost, e->stream);
    if (r != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("step (exchange pack): ") + hipGetErrorString(r));
    e->auto_round = e->round;
  }
  const bool cnt_lost = count_lost_on(e);
  if (cnt_lost) {  // this round's lost sends: the next round's arrivals are its sends minus them
    hipError_t x = enqueue_lost_count(e, g, graph_for_arrivals(e, e->round), e->round);
    if (x != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("step (lost sends): ") + hipGetErrorString(x));
  }
  if ((rc = read_stats())) return rc;
  std::memcpy(e->stats_base, e->h_stats, sizeof(e->stats_base));  // the next round counts from here
  if ((rc = check_scatter_list(e, e->h_stats[STAT_COUNT]))) return rc;
  if (e->auto_round == e->round)  // the round's own pack landed with its counters
    for (int q = 0; q + 1 < (int)e->send_seg.size(); ++q) e->auto_cnt[q] = (int64_t)e->h_seg_cnt[q];
#ifdef P2PG_PROF
  if (fused_round && s.prof && std::getenv("P2PG_PROF_ROUNDS")) {
    // development builds: per-round fused-kernel segment clocks (then reset)
    unsigned long long h[9];
    HIPCHK(e, hipMemcpy(h, s.prof, sizeof(h), hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemset(s.prof, 0, sizeof(h)));
    fprintf(stderr, "P2PG_PROF_ROUND %d", e->round);
    for (int i = 0; i < 9; ++i) fprintf(stderr, " %llu", h[i]);
    fprintf(stderr, "\n");
  }
#endif
  const bool active = tot[ST_NEW] != 0;
  e->frontier_kept_prev = e->frontier_kept;
  e->frontier_kept = !(((fused_round || up_round) && !p.store_f) || p.store_f == 2) || !active;
  if (out) {
    out->round = e->round;
    out->active = active ? 1 : 0;
    out->new_deliveries = tot[ST_NEW];
    out->relays = tot[ST_RELAYS];
    out->active_vertices = tot[ST_ACTIVE_V];
    out->active_words = tot[ST_ACTIVE_W];
    out->wedges = tot[ST_WEDGES];
    out->deg_active = tot[ST_DEG_ACT];
    out->scatter_words = tot[ST_SCATTER];
    out->touched_words = tot[ST_AUX];
    out->push_form = !gossip ? P2PG_PUSH_NONE
                     : fused_round ? P2PG_PUSH_FUSED
                     : up_round ? P2PG_PUSH_UPDATE_EDGE
                     : e->last_push_e ? P2PG_PUSH_EDGE : P2PG_PUSH_ATOMIC;
    out->received_exact = received_exact(e) ? 1 : 0;
    out->received = e->round == 0 ? 0 : e->sent_last - e->lost_last;
  }
  e->sent_last = tot[ST_RELAYS];
  e->lost_last = cnt_lost ? (uint64_t)e->h_cnt2[1] : 0;
  e->total_relays += tot[ST_RELAYS];
  e->prev2_aw = e->prev_aw;
  e->prev2_av = e->prev_av;
  e->prev2_new = e->last_new;
  e->prev_aw = tot[ST_ACTIVE_W];
  e->prev_av = tot[ST_ACTIVE_V];
  e->last_new = tot[ST_NEW];
  e->prev_sw = tot[ST_SCATTER];
  if (e->last_push_e) e->saw_dense = true;
  e->round += 1;
  if (!active && !(e->cfg.flags & P2PG_FLAG_NO_AUTOSTOP)) e->done = true;
  return active ? 1 : 0;
}

int p2pg_step_end(p2pg_engine* e, p2pg_round_stats* out) { return p2pg_step(e, out); }

// p2pg_run's decay phase: after the dense rounds, while receipts shrink, every round is an update
// of the row pushes and a row-atomic push whose form, list bound (the last round's pushed masks,
// shrinking too) and dedup setting need none of its own counters -- so BATCH_MAX of them are
// enqueued at once, each writing its counters to its own slot, and read with ONE host
// synchronisation (c4: ~20 tail rounds of 0.05-0.2 ms kernels each paid a full host round trip).
// Rounds enqueued after the run went quiet see an empty frontier and change nothing; they are
// not reported and the engine stands where p2pg_step would have left it.  The list is sized by
// a bound that holds for the batch's first round (its frontier words <= the masks pushed into it,
// prev_sw) with room to spare for the others (decay: each round's frontier is ~2.5x smaller); a
// later round whose frontier still outgrew it had its push truncated, so the call reports the
// rounds before that one, fails (P2PG_ERR_STATE) and leaves the engine refusing every further
// round until a reset (the device state past that round is not the run's).
constexpr int BATCH_MAX = 8;

static bool decay_batchable(const p2pg_engine* e) {
  const int br = e->batch_rounds < 0 ? BATCH_MAX : e->batch_rounds;
  return br > 1 && e->have_state && !e->done && !e->begun && e->round > 0 && !count_lost_on(e) &&
         e->cfg.mode == P2PG_MODE_GOSSIP && e->saw_dense && !e->last_push_e &&
         e->last_new < e->prev2_new && e->prev_sw > 0 && !e->consume_next && e->arr_round < 0 &&
         !e->d_gid && !(e->cfg.flags & P2PG_FLAG_NO_AUTOSTOP) && e->push_mode != 2 &&
         e->auto_buf == nullptr && sparse_scatter_on(e) &&
         e->last_new * 16 < (uint64_t)e->V;  // the tail: small rounds, where the syncs dominate
}

// n_left: rounds the p2pg_run call may still run (its last two keep their frontier rows whole).
static int run_decay_batch(p2pg_engine* e, int32_t R, p2pg_round_stats* out, int32_t* ran,
                           int32_t n_left) {
  constexpr size_t SLOT = STAT_COUNT + 1;  // counters + the sparse list's fill count
  DevState& s = e->st;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  if (!e->d_bstats) {
    HIPCHK(e, hipMalloc((void**)&e->d_bstats, sizeof(unsigned long long) * SLOT * BATCH_MAX));
    HIPCHK(e, hipHostMalloc((void**)&e->h_bstats, sizeof(unsigned long long) * SLOT * BATCH_MAX));
  }
  HIPCHK(e, hipMemsetAsync(e->d_bstats, 0, sizeof(unsigned long long) * SLOT * R, e->stream));
  // the list, sized once for the batch: the first round's bound, doubled for the others
  SparseBufs b;
  hipError_t lr = sparse_bufs(e, 2 * (int64_t)e->prev_sw, b);
  if (lr != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("run (batch list): ") + hipGetErrorString(lr));
  const uint64_t words = (uint64_t)e->wlist_cap;  // no round of the batch grows the list
  unsigned long long* const stats0 = s.stats;
  const DevGraph g = graph(e);
  int rc = P2PG_OK;
  bool partial[BATCH_MAX] = {false};
  for (int32_t i = 0; i < R && rc == P2PG_OK; ++i) {
    s.stats = e->d_bstats + SLOT * i;
    RoundParams p = params(e);
    p.round = e->round + i;
    if (partial_frontier(e, i + 2 < n_left)) p.store_f = 2;
    partial[i] = p.store_f == 2;
    rc = timed(e, 4, [&] { return launch_gossip_update(g, s, p, e->stream); });
    if (rc == P2PG_OK && s.hop) rc = timed(e, 3, [&] { return launch_record(g, s, p, e->stream); });
    p.dedup_push = e->push_dedup != 0;  // decay phase (saw_dense: the rule of p2pg_step)
    if (rc == P2PG_OK)
      rc = timed(e, 2, [&] {
        return launch_scatter_atomic(e, g, p, std::min<uint64_t>(e->prev_sw, words));
      });
  }
  s.stats = stats0;
  e->wlist_check = false;
  if (rc) return rc;
  HIPCHK(e, hipMemcpyAsync(e->h_bstats, e->d_bstats, sizeof(unsigned long long) * SLOT * R,
                           hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, round_sync(e));
  if ((rc = resolve_timings(e))) return rc;
  *ran = 0;
  for (int32_t i = 0; i < R; ++i) {
    const unsigned long long* h = e->h_bstats + SLOT * i;
    if ((int64_t)h[STAT_COUNT] > e->wlist_cap) {
      // round e->round's push was truncated: the rounds before it stand (reported), nothing after
      e->failed = "round " + std::to_string(e->round) + " of a batched decay run outgrew its sparse push list (" +
                  std::to_string(h[STAT_COUNT]) + " words listed, room for " + std::to_string(e->wlist_cap) +
                  "); reset to run again";
      e->done = true;
      return fail(e, P2PG_ERR_STATE, "run: " + e->failed);
    }
    uint64_t tot[STAT_N] = {0};
    for (int sh = 0; sh < STAT_SHARDS; ++sh)
      for (int q = 0; q < STAT_N; ++q) tot[q] += h[sh * STAT_N + q];
    const bool active = tot[ST_NEW] != 0;
    p2pg_round_stats& o = out[i];
    o.round = e->round;
    o.active = active ? 1 : 0;
    o.new_deliveries = tot[ST_NEW];
    o.relays = tot[ST_RELAYS];
    o.active_vertices = tot[ST_ACTIVE_V];
    o.active_words = tot[ST_ACTIVE_W];
    o.wedges = tot[ST_WEDGES];
    o.deg_active = tot[ST_DEG_ACT];
    o.scatter_words = tot[ST_SCATTER];
    o.touched_words = tot[ST_AUX];
    o.push_form = P2PG_PUSH_ATOMIC;
    o.received_exact = received_exact(e) ? 1 : 0;
    o.received = e->round == 0 ? 0 : e->sent_last - e->lost_last;
    e->sent_last = tot[ST_RELAYS];
    e->lost_last = 0;  // (no churn in a batched run)
    e->total_relays += tot[ST_RELAYS];
    e->frontier_kept_prev = e->frontier_kept;
    e->frontier_kept = !(partial[i] && active);
    e->prev2_aw = e->prev_aw;
    e->prev2_av = e->prev_av;
    e->prev2_new = e->last_new;
    e->prev_aw = tot[ST_ACTIVE_W];
    e->prev_av = tot[ST_ACTIVE_V];
    e->last_new = tot[ST_NEW];
    e->prev_sw = tot[ST_SCATTER];
    e->round += 1;
    *ran = i + 1;
    if (!active) {
      e->done = true;  // (rounds enqueued after this one saw an empty frontier)
      break;
    }
  }
  return P2PG_OK;
}

int p2pg_run(p2pg_engine* e, int32_t max_rounds, p2pg_round_stats* per_round,
             int32_t* n_rounds) {
  if (!e) return P2PG_ERR_ARG;
  int32_t n = 0;
  int rc = 1;
  while (n < max_rounds) {
    p2pg_round_stats tmp;
    if (decay_batchable(e) && max_rounds - n >= 2) {
      const int br = e->batch_rounds < 0 ? BATCH_MAX : std::min(e->batch_rounds, BATCH_MAX);
      const int32_t R = std::min<int32_t>(br, max_rounds - n);
      p2pg_round_stats buf[BATCH_MAX];
      int32_t ran = 0;
      rc = run_decay_batch(e, R, buf, &ran, max_rounds - n);
      if (per_round) std::memcpy(per_round + n, buf, sizeof(p2pg_round_stats) * ran);
      n += ran;
      if (rc < 0) {  // (the rounds that stand are reported)
        if (n_rounds) *n_rounds = n;
        return rc;
      }
      rc = e->done ? 0 : 1;
      if (rc == 0) break;
      continue;
    }
    // only the last two rounds a call may run can leave frontiers behind for the caller (the
    // deliveries of the last round and their parents in the round before; snapshots); a
    // quiescent round has none
    e->skip_frontier = n + 2 < max_rounds && !count_lost_on(e);  // (the lost count reads F)
    rc = p2pg_step(e, per_round ? &per_round[n] : &tmp);
    e->skip_frontier = false;
    if (rc < 0) return rc;
    ++n;
    if (rc == 0) break;
  }
  if (n_rounds) *n_rounds = n;
  return rc;
}

int p2pg_get_new_deliveries(p2pg_engine* e, int64_t cap, int32_t* peer, int32_t* msg,
                            int32_t* hop, int32_t* parent, int64_t* n_out) {
  if (!e || cap < 0 || !n_out || (cap > 0 && (!peer || !msg || !hop || !parent)))
    return fail(e, P2PG_ERR_ARG, "get_new_deliveries: bad arguments");
  if (!e->have_state || e->round == 0)
    return fail(e, P2PG_ERR_STATE, "get_new_deliveries: no round has run");
  if (e->last_new == 0) {  // a round without receipts has no deliveries (and needs no parents)
    *n_out = 0;
    return P2PG_OK;
  }
  if (!e->frontier_kept)
    return fail(e, P2PG_ERR_STATE, "get_new_deliveries: the last round's frontier was not kept");
  if (!e->frontier_kept_prev)
    return fail(e, P2PG_ERR_STATE, "get_new_deliveries: the parents need the frontier of the round "
                                   "before, which was not kept (a fused round inside p2pg_run, or "
                                   "the round a snapshot was restored at)");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  // the most recent round is e->round - 1; its frontier is F[(round-1)&1]
  RoundParams p = params(e);
  p.round = e->round - 1;
  const DevGraph g = graph_for_arrivals(e, p.round);
  int32_t *dpeer = nullptr, *dmsg = nullptr, *dpar = nullptr;
  unsigned long long* dcnt = nullptr;
  const int64_t c = cap > 0 ? cap : 1;
  HIPCHK(e, hipMalloc((void**)&dpeer, sizeof(int32_t) * c));
  HIPCHK(e, hipMalloc((void**)&dmsg, sizeof(int32_t) * c));
  HIPCHK(e, hipMalloc((void**)&dpar, sizeof(int32_t) * c));
  HIPCHK(e, hipMalloc((void**)&dcnt, sizeof(unsigned long long)));
  HIPCHK(e, hipMemsetAsync(dcnt, 0, sizeof(unsigned long long), e->stream));
  hipError_t lr = launch_deliveries(g, e->st, p, cap, dpeer, dmsg, dpar, dcnt, e->stream);
  unsigned long long cnt = 0;
  if (lr == hipSuccess) lr = hipMemcpyAsync(&cnt, dcnt, sizeof(cnt), hipMemcpyDeviceToHost, e->stream);
  if (lr == hipSuccess) lr = hipStreamSynchronize(e->stream);
  const int64_t n = std::min<int64_t>((int64_t)cnt, cap);
  std::vector<int32_t> hp(n), hm(n), hpar(n);
  if (lr == hipSuccess && n > 0) {
    lr = hipMemcpy(hp.data(), dpeer, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
    if (lr == hipSuccess) lr = hipMemcpy(hm.data(), dmsg, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
    if (lr == hipSuccess) lr = hipMemcpy(hpar.data(), dpar, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
  }
  (void)hipFree(dpeer);
  (void)hipFree(dmsg);
  (void)hipFree(dpar);
  (void)hipFree(dcnt);
  if (lr != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("get_new_deliveries: ") + hipGetErrorString(lr));
  // deterministic order: ascending (peer, msg)  (the compat layer replays hooks in it)
  std::vector<int64_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
    return hp[a] != hp[b] ? hp[a] < hp[b] : hm[a] < hm[b];
  });
  const bool map = !e->h_gid.empty();
  for (int64_t i = 0; i < n; ++i) {
    const int32_t pr = hpar[idx[i]];
    peer[i] = map ? e->h_gid[hp[idx[i]]] : hp[idx[i]];
    msg[i] = hm[idx[i]];
    hop[i] = p.round;
    parent[i] = (map && pr >= 0) ? e->h_gid[pr] : pr;
  }
  *n_out = (int64_t)cnt;
  return P2PG_OK;
}

// Shared preconditions of the sends stream / relay withdrawal: a round ran, its frontier (and,
// flood, the one before it: the senders' parents) is in F, and no topology update or half
// round stands between that round and now.
static int sends_state(p2pg_engine* e, const char* what) {
  const std::string w(what);
  if (!e->have_state || e->round == 0) return fail(e, P2PG_ERR_STATE, w + ": no round has run");
  if (e->begun) return fail(e, P2PG_ERR_STATE, w + ": a round has begun (step_begin)");
  if (e->arr_round >= 0 && e->arr_round == e->round)
    return fail(e, P2PG_ERR_STATE, w + ": the connections changed since the round (call it before p2pg_update_edges)");
  if (e->last_new == 0) return P2PG_OK;
  if (!e->frontier_kept) return fail(e, P2PG_ERR_STATE, w + ": the last round's frontier was not kept");
  if (e->cfg.mode == P2PG_MODE_FLOOD && e->round > 1 && !e->frontier_kept_prev)
    return fail(e, P2PG_ERR_STATE, w + ": the senders' parents need the frontier of the round before, "
                                       "which was not kept");
  return P2PG_OK;
}

int p2pg_get_sends(p2pg_engine* e, int64_t cap, int32_t* sender, int32_t* receiver, int32_t* msg,
                   uint8_t* lost, int64_t* n_out) {
  if (!e || cap < 0 || !n_out || (cap > 0 && (!sender || !receiver || !msg || !lost)))
    return fail(e, P2PG_ERR_ARG, "get_sends: bad arguments");
  int rc = sends_state(e, "get_sends");
  if (rc) return rc;
  if (e->last_new == 0) {
    *n_out = 0;
    return P2PG_OK;
  }
  HIPCHK(e, hipSetDevice(e->cfg.device));
  const int32_t r = e->round - 1;
  RoundParams p = params(e);
  p.round = r;
  const int64_t c = cap > 0 ? cap : 1;
  int32_t *ds = nullptr, *dr = nullptr, *dm = nullptr;
  uint8_t* dl = nullptr;
  HIPCHK(e, hipMalloc((void**)&ds, sizeof(int32_t) * c));
  HIPCHK(e, hipMalloc((void**)&dr, sizeof(int32_t) * c));
  HIPCHK(e, hipMalloc((void**)&dm, sizeof(int32_t) * c));
  HIPCHK(e, hipMalloc((void**)&dl, c));
  hipError_t lr = hipMemsetAsync(e->d_cnt2, 0, 2 * sizeof(unsigned long long), e->stream);
  if (lr == hipSuccess)
    lr = launch_sends(graph(e), graph_for_arrivals(e, r), e->st, p, true, cap, ds, dr, dm, dl, e->d_cnt2, e->stream);
  unsigned long long cnt = 0;
  if (lr == hipSuccess) lr = hipMemcpyAsync(&cnt, e->d_cnt2, sizeof(cnt), hipMemcpyDeviceToHost, e->stream);
  if (lr == hipSuccess) lr = hipStreamSynchronize(e->stream);
  const int64_t n = std::min<int64_t>((int64_t)cnt, cap);
  std::vector<int32_t> hs(n), hr(n), hm(n);
  std::vector<uint8_t> hl(n);
  if (lr == hipSuccess && n > 0) {
    lr = hipMemcpy(hs.data(), ds, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
    if (lr == hipSuccess) lr = hipMemcpy(hr.data(), dr, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
    if (lr == hipSuccess) lr = hipMemcpy(hm.data(), dm, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
    if (lr == hipSuccess) lr = hipMemcpy(hl.data(), dl, n, hipMemcpyDeviceToHost);
  }
  (void)hipFree(ds);
  (void)hipFree(dr);
  (void)hipFree(dm);
  (void)hipFree(dl);
  if (lr != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("get_sends: ") + hipGetErrorString(lr));
  // deterministic order: ascending (receiver, sender, msg) -- the harness's delivery order up to the
  // order of one sender's packets on one connection, which the caller knows (its relay order)
  std::vector<int64_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
    if (hr[a] != hr[b]) return hr[a] < hr[b];
    return hs[a] != hs[b] ? hs[a] < hs[b] : hm[a] < hm[b];
  });
  const bool map = !e->h_gid.empty();
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = idx[i];
    sender[i] = map ? e->h_gid[hs[k]] : hs[k];
    receiver[i] = map ? e->h_gid[hr[k]] : hr[k];
    msg[i] = hm[k];
    lost[i] = hl[k];
  }
  *n_out = (int64_t)cnt;
  return P2PG_OK;
}

int p2pg_drop_relays(p2pg_engine* e, int64_t n, const int32_t* peer, const int32_t* msg) {
  if (!e || n < 0 || (n > 0 && (!peer || !msg))) return fail(e, P2PG_ERR_ARG, "drop_relays: bad arguments");
  int rc = sends_state(e, "drop_relays");
  if (rc) return rc;
  if (n == 0) return P2PG_OK;
  if (e->d_gid || (e->cfg.flags & P2PG_FLAG_LOCAL_GRAPH))
    return fail(e, P2PG_ERR_STATE, "drop_relays: not on a vertex-partitioned rank");
  const bool gossip = e->cfg.mode == P2PG_MODE_GOSSIP;
  if (!gossip && e->consume_next)
    return fail(e, P2PG_ERR_STATE, "drop_relays: the last round's sends were materialized (restored snapshot)");
  std::vector<uint64_t> list(n);
  for (int64_t i = 0; i < n; ++i) {
    if (peer[i] < 0 || peer[i] >= e->V || msg[i] < 0 || msg[i] >= e->M)
      return fail(e, P2PG_ERR_ARG, "drop_relays: peer or message out of range");
    list[i] = ((uint64_t)(uint32_t)peer[i] << 32) | (uint32_t)msg[i];
  }
  std::sort(list.begin(), list.end());
  if (std::adjacent_find(list.begin(), list.end()) != list.end())
    return fail(e, P2PG_ERR_ARG, "drop_relays: a first receipt is listed twice");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  const int32_t r = e->round - 1;
  uint64_t* dl = nullptr;
  HIPCHK(e, hipMalloc((void**)&dl, sizeof(uint64_t) * n));
  hipError_t lr = hipMemcpyAsync(dl, list.data(), sizeof(uint64_t) * n, hipMemcpyHostToDevice, e->stream);
  if (lr == hipSuccess) lr = hipMemsetAsync(e->d_cnt2, 0, 2 * sizeof(unsigned long long), e->stream);
  if (lr == hipSuccess) lr = launch_drop(e->st, r, dl, n, true, e->d_cnt2, e->stream);
  if (lr == hipSuccess)
    lr = hipMemcpyAsync(e->h_cnt2, e->d_cnt2, sizeof(unsigned long long), hipMemcpyDeviceToHost, e->stream);
  if (lr == hipSuccess) lr = hipStreamSynchronize(e->stream);
  if (lr == hipSuccess && (int64_t)e->h_cnt2[0] != n) {
    (void)hipFree(dl);
    return fail(e, P2PG_ERR_ARG, "drop_relays: " + std::to_string(n - (int64_t)e->h_cnt2[0]) +
                                     " listed (peer, msg) are not first receipts of the last round");
  }
  if (lr == hipSuccess) lr = launch_drop(e->st, r, dl, n, false, nullptr, e->stream);
  if (lr == hipSuccess) lr = launch_rebuild_aw(e->st, r, e->V, e->stream);
  // the relays these receipts would have made (node.py:106-116): flood every connection but
  // the sender (all of them at the origin), gossip min(k, deg)
  uint64_t cancelled = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t v = (int64_t)(list[i] >> 32);
    const uint64_t deg = (uint64_t)(e->h_rowptr[v + 1] - e->h_rowptr[v]);
    cancelled += gossip ? std::min<uint64_t>(deg, (uint64_t)e->cfg.fanout) : (r == 0 ? deg : (deg ? deg - 1 : 0));
  }
  if (lr == hipSuccess && gossip) {
    // this round's pushes left inside the round: push the remaining receipts again, as row
    // atomics, into the cleared row-push planes the next round consumes (the Philox picks are a
    // pure function of round, peer and message, so the others go where they went)
    DevState& s = e->st;
    const int nx = e->round & 1;
    lr = hipMemsetAsync(s.next[nx], 0, e->plane_bytes, e->stream);
    if (lr == hipSuccess) lr = hipMemsetAsync(s.T[nx], 0, e->bm_bytes, e->stream);
    RoundParams p = params(e);
    p.round = r;
    if (lr == hipSuccess) lr = launch_scatter_atomic(e, graph(e), p, std::max<uint64_t>(e->prev_aw, 1));
  }
  if (lr == hipSuccess && count_lost_on(e))
    lr = enqueue_lost_count(e, graph(e), graph_for_arrivals(e, r), r);
  if (lr == hipSuccess) lr = hipStreamSynchronize(e->stream);
  (void)hipFree(dl);
  if (lr != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("drop_relays: ") + hipGetErrorString(lr));
  if (gossip) {
    if (e->wlist_check) {
      unsigned long long listed = 0;
      HIPCHK(e, hipMemcpy(&listed, e->st.stats + STAT_COUNT, sizeof(listed), hipMemcpyDeviceToHost));
      if ((rc = check_scatter_list(e, listed))) return rc;
    }
    e->consume_next = true;
    e->last_push_e = false;
    e->stats_clear = true;  // the re-push counted into the round counters
  }
  if (count_lost_on(e)) e->lost_last = (uint64_t)e->h_cnt2[1];
  e->sent_last -= std::min(cancelled, e->sent_last);
  e->total_relays -= std::min(cancelled, e->total_relays);
  return P2PG_OK;
}

int p2pg_read_planes(p2pg_engine* e, uint64_t* seen, int32_t* hop, int32_t* parent) {
  if (!e || !e->have_state) return fail(e, P2PG_ERR_STATE, "read_planes: no state");
  if ((hop || parent) && !e->st.hop)
    return fail(e, P2PG_ERR_STATE, "read_planes: hop/parent need P2PG_FLAG_RECORD");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (seen) HIPCHK(e, hipMemcpy(seen, e->st.seen, e->plane_bytes, hipMemcpyDeviceToHost));
  const size_t hb = (size_t)e->V * e->M * sizeof(int32_t);
  if (hop) HIPCHK(e, hipMemcpy(hop, e->st.hop, hb, hipMemcpyDeviceToHost));
  if (parent) {
    HIPCHK(e, hipMemcpy(parent, e->st.parent, hb, hipMemcpyDeviceToHost));
    if (!e->h_gid.empty())  // local -> global sender ids
      for (size_t i = 0; i < (size_t)e->V * e->M; ++i)
        if (parent[i] >= 0) parent[i] = e->h_gid[parent[i]];
  }
  return P2PG_OK;
}

int p2pg_read_seen_word(p2pg_engine* e, int32_t w, uint64_t* out) {
  if (!e || !e->have_state) return fail(e, P2PG_ERR_STATE, "read_seen_word: no state");
  if (w < 0 || w >= e->W || !out) return fail(e, P2PG_ERR_ARG, "read_seen_word: word out of range");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  // column w of the [V][W] plane gathered into a contiguous device buffer, then one copy
  uint64_t* col = nullptr;
  HIPCHK(e, hipMalloc((void**)&col, sizeof(uint64_t) * (size_t)e->V));
  hipError_t r = launch_column(e->st.seen, e->W, w, e->V, col, e->stream);
  if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
  if (r == hipSuccess) r = hipMemcpy(out, col, sizeof(uint64_t) * (size_t)e->V, hipMemcpyDeviceToHost);
  (void)hipFree(col);
  if (r != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("read_seen_word: ") + hipGetErrorString(r));
  return P2PG_OK;
}

int p2pg_set_global_ids(p2pg_engine* e, const int32_t* gid) {
  if (!e || !e->d_rowptr) return fail(e, P2PG_ERR_STATE, "set_global_ids: load a graph first");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  dfree(e->d_gid);
  e->h_gid.clear();
  if (!gid) return P2PG_OK;
  for (int64_t v = 1; v < e->V; ++v)
    if (gid[v] <= gid[v - 1])
      return fail(e, P2PG_ERR_ARG, "set_global_ids: ids must be strictly ascending (global order)");
  e->h_gid.assign(gid, gid + e->V);
  HIPCHK(e, hipMalloc((void**)&e->d_gid, sizeof(int32_t) * e->V));
  HIPCHK(e, hipMemcpy(e->d_gid, gid, sizeof(int32_t) * e->V, hipMemcpyHostToDevice));
  return P2PG_OK;
}

int p2pg_set_ghost_senders(p2pg_engine* e, const int32_t* ghost_deg, const int32_t* slot_pos) {
  if (!e || !e->d_rowptr) return fail(e, P2PG_ERR_STATE, "set_ghost_senders: load a graph first");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  dfree(e->d_gdeg);
  dfree(e->d_gpos);
  if (!ghost_deg && !slot_pos) return P2PG_OK;
  if (!ghost_deg || !slot_pos) return fail(e, P2PG_ERR_ARG, "set_ghost_senders: need both arrays");
  for (int64_t v = 0; v < e->V; ++v)
    for (int64_t j = e->h_rowptr[v]; j < e->h_rowptr[v + 1]; ++j) {
      const int32_t u = e->h_colidx[j];
      if (slot_pos[j] < -1 || (slot_pos[j] >= 0 && slot_pos[j] >= ghost_deg[u]))
        return fail(e, P2PG_ERR_ARG, "set_ghost_senders: slot position outside the ghost's row");
    }
  HIPCHK(e, hipMalloc((void**)&e->d_gdeg, sizeof(int32_t) * (size_t)e->V));
  HIPCHK(e, hipMalloc((void**)&e->d_gpos, sizeof(int32_t) * (size_t)(e->nnz ? e->nnz : 1)));
  HIPCHK(e, hipMemcpy(e->d_gdeg, ghost_deg, sizeof(int32_t) * (size_t)e->V, hipMemcpyHostToDevice));
  if (e->nnz)
    HIPCHK(e, hipMemcpy(e->d_gpos, slot_pos, sizeof(int32_t) * (size_t)e->nnz, hipMemcpyHostToDevice));
  return P2PG_OK;
}

int p2pg_set_exchange(p2pg_engine* e, int64_t n_send, const int32_t* send_local, int64_t n_recv,
                      const int32_t* recv_local) {
  if (!e || !e->d_rowptr || n_send < 0 || n_recv < 0 || (n_send && !send_local) ||
      (n_recv && !recv_local))
    return fail(e, P2PG_ERR_ARG, "set_exchange: bad arguments");
  if (e->begun) return fail(e, P2PG_ERR_STATE, "set_exchange: a round has begun (step_begin)");
  for (int64_t i = 0; i < n_send; ++i)
    if (send_local[i] < 0 || send_local[i] >= e->V) return fail(e, P2PG_ERR_ARG, "set_exchange: send id out of range");
  for (int64_t i = 0; i < n_recv; ++i)
    if (recv_local[i] < 0 || recv_local[i] >= e->V) return fail(e, P2PG_ERR_ARG, "set_exchange: recv id out of range");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  dfree(e->d_send);
  dfree(e->d_recv);
  e->n_send = n_send;
  e->n_recv = n_recv;
  HIPCHK(e, hipMalloc((void**)&e->d_send, sizeof(int32_t) * (n_send ? n_send : 1)));
  HIPCHK(e, hipMalloc((void**)&e->d_recv, sizeof(int32_t) * (n_recv ? n_recv : 1)));
  if (n_send) HIPCHK(e, hipMemcpy(e->d_send, send_local, sizeof(int32_t) * n_send, hipMemcpyHostToDevice));
  if (n_recv) HIPCHK(e, hipMemcpy(e->d_recv, recv_local, sizeof(int32_t) * n_recv, hipMemcpyHostToDevice));
  // border peers: a ghost (recv list) among the neighbours -- their pull / update waits for the
  // exchanged rows (phase 1); every other peer can run while the exchange is in flight
  dfree(e->d_border);
  if (n_recv) {
    std::vector<uint8_t> ghost((size_t)e->V, 0);
    for (int64_t i = 0; i < n_recv; ++i) ghost[recv_local[i]] = 1;
    std::vector<uint32_t> border((size_t)((e->V + 31) / 32), 0u);
    for (int64_t v = 0; v < e->V; ++v)
      for (int64_t j = e->h_rowptr[v]; j < e->h_rowptr[v + 1]; ++j)
        if (ghost[e->h_colidx[j]]) {
          border[v >> 5] |= 1u << (v & 31);
          break;
        }
    HIPCHK(e, hipMalloc((void**)&e->d_border, sizeof(uint32_t) * border.size()));
    HIPCHK(e, hipMemcpy(e->d_border, border.data(), sizeof(uint32_t) * border.size(), hipMemcpyHostToDevice));
  }
  return P2PG_OK;
}

int p2pg_set_exchange_segments(p2pg_engine* e, int32_t nseg, const int64_t* send_counts,
                               const int64_t* recv_counts) {
  if (!e || !e->d_send || nseg < 1 || nseg > P2PG_MAX_RANKS || !send_counts || !recv_counts)
    return fail(e, P2PG_ERR_ARG, "set_exchange_segments: bad arguments (set_exchange first; 1..16 ranks)");
  std::vector<int64_t> so(nseg + 1, 0), ro(nseg + 1, 0);
  for (int q = 0; q < nseg; ++q) {
    if (send_counts[q] < 0 || recv_counts[q] < 0) return fail(e, P2PG_ERR_ARG, "set_exchange_segments: negative count");
    so[q + 1] = so[q] + send_counts[q];
    ro[q + 1] = ro[q] + recv_counts[q];
  }
  if (so[nseg] != e->n_send || ro[nseg] != e->n_recv)
    return fail(e, P2PG_ERR_ARG, "set_exchange_segments: counts do not add up to the exchange lists");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  dfree(e->d_send_seg);
  dfree(e->d_recv_seg);
  dfree(e->d_seg_cnt);
  if (e->h_seg_cnt) (void)hipHostFree(e->h_seg_cnt);
  e->h_seg_cnt = nullptr;
  e->send_seg = so;
  e->recv_seg = ro;
  HIPCHK(e, hipMalloc((void**)&e->d_send_seg, sizeof(int64_t) * so.size()));
  HIPCHK(e, hipMalloc((void**)&e->d_recv_seg, sizeof(int64_t) * ro.size()));
  HIPCHK(e, hipMemcpy(e->d_send_seg, so.data(), sizeof(int64_t) * so.size(), hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(e->d_recv_seg, ro.data(), sizeof(int64_t) * ro.size(), hipMemcpyHostToDevice));
  HIPCHK(e, hipMalloc((void**)&e->d_seg_cnt, sizeof(unsigned long long) * P2PG_MAX_RANKS));
  HIPCHK(e, hipHostMalloc((void**)&e->h_seg_cnt, sizeof(unsigned long long) * P2PG_MAX_RANKS));
  return P2PG_OK;
}

int p2pg_set_exchange_buffer(p2pg_engine* e, int32_t plane, void* dev_buf) {
  if (!e) return P2PG_ERR_ARG;
  if (!dev_buf) {
    e->auto_buf = nullptr;
    e->auto_plane = -1;
    e->auto_round = -1;
    return P2PG_OK;
  }
  if (plane != 0 && plane != 1) return fail(e, P2PG_ERR_ARG, "set_exchange_buffer: plane 0 or 1");
  if (!e->d_seg_cnt) return fail(e, P2PG_ERR_STATE, "set_exchange_buffer: set_exchange_segments first");
  if (plane == 1 && e->cfg.mode != P2PG_MODE_GOSSIP)
    return fail(e, P2PG_ERR_ARG, "set_exchange_buffer: plane 1 is for gossip pushes");
  if (e->begun) return fail(e, P2PG_ERR_STATE, "set_exchange_buffer: a round has begun (step_begin)");
  e->auto_buf = dev_buf;
  e->auto_plane = plane;
  e->auto_round = -1;
  return P2PG_OK;
}

int p2pg_exchange_pack_live(p2pg_engine* e, int32_t plane, void* dev_buf, int64_t* counts) {
  if (!e || !e->have_state || e->round == 0 || (plane != 0 && plane != 1) || !dev_buf || !counts)
    return fail(e, P2PG_ERR_STATE, "exchange_pack_live: need a completed round, plane 0 or 1, buffers");
  if (!e->d_seg_cnt) return fail(e, P2PG_ERR_STATE, "exchange_pack_live: set_exchange_segments first");
  if (e->begun) return fail(e, P2PG_ERR_STATE, "exchange_pack_live: the next round has begun");
  if (plane == 1 && e->cfg.mode != P2PG_MODE_GOSSIP)
    return fail(e, P2PG_ERR_ARG, "exchange_pack_live: plane 1 is for gossip pushes");
  const int nseg = (int)e->send_seg.size() - 1;
  if (dev_buf == e->auto_buf && plane == e->auto_plane && e->auto_round == e->round - 1) {
    // packed by the round itself (p2pg_set_exchange_buffer), counts read with its counters
    for (int q = 0; q < nseg; ++q) counts[q] = e->auto_cnt[q];
    e->auto_round = -1;  // handed over once
    return P2PG_OK;
  }
  HIPCHK(e, hipSetDevice(e->cfg.device));
  // plane 0 moves frontier rows owner -> ghost (send list); plane 1 pushes ghost -> owner
  const bool fwd = plane == 0;
  const int32_t* ids = fwd ? e->d_send : e->d_recv;
  const int64_t n = fwd ? e->n_send : e->n_recv;
  const int64_t* seg = fwd ? e->d_send_seg : e->d_recv_seg;
  HIPCHK(e, hipMemsetAsync(e->d_seg_cnt, 0, sizeof(unsigned long long) * P2PG_MAX_RANKS, e->stream));
  hipError_t r = launch_pack_live(e->st, plane, e->round - 1, ids, n, seg, nseg, e->d_seg_cnt,
                                  (int64_t*)dev_buf, e->stream);
  if (r == hipSuccess)
    r = hipMemcpyAsync(e->h_seg_cnt, e->d_seg_cnt, sizeof(unsigned long long) * nseg, hipMemcpyDeviceToHost,
                       e->stream);
  if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
  if (r != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("exchange_pack_live: ") + hipGetErrorString(r));
  for (int q = 0; q < nseg; ++q) counts[q] = (int64_t)e->h_seg_cnt[q];
  return P2PG_OK;
}

int p2pg_exchange_unpack_live(p2pg_engine* e, int32_t plane, const void* dev_buf, const int64_t* counts) {
  if (!e || !e->have_state || e->round == 0 || (plane != 0 && plane != 1) || !counts)
    return fail(e, P2PG_ERR_STATE, "exchange_unpack_live: need a completed round, plane 0 or 1, counts");
  if (!e->d_seg_cnt) return fail(e, P2PG_ERR_STATE, "exchange_unpack_live: set_exchange_segments first");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  const int nseg = (int)e->send_seg.size() - 1;
  const bool fwd = plane == 0;  // plane 0 lands in the recv list (ghosts), plane 1 in the send list
  const int32_t* ids = fwd ? e->d_recv : e->d_send;
  const std::vector<int64_t>& lst = fwd ? e->recv_seg : e->send_seg;
  const int64_t* lseg = fwd ? e->d_recv_seg : e->d_send_seg;
  int64_t ro[P2PG_MAX_RANKS + 1] = {0};
  for (int q = 0; q < nseg; ++q) {
    if (counts[q] < 0 || counts[q] > lst[q + 1] - lst[q])
      return fail(e, P2PG_ERR_ARG, "exchange_unpack_live: more records than the list segment holds");
    ro[q + 1] = ro[q] + counts[q];
  }
  if (ro[nseg] > 0 && !dev_buf) return fail(e, P2PG_ERR_ARG, "exchange_unpack_live: no buffer");
  // asynchronous on the engine stream: the next step orders after it
  hipError_t r = launch_unpack_live(e->st, plane, e->round - 1, ids, lseg, nseg, ro, (const int64_t*)dev_buf,
                                    e->stream);
  if (r != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("exchange_unpack_live: ") + hipGetErrorString(r));
  return P2PG_OK;
}

static int exchange(p2pg_engine* e, int32_t plane, bool pack, void* buf) {
  if (!e || !e->have_state || e->round == 0 || (plane != 0 && plane != 1))
    return fail(e, P2PG_ERR_STATE, "exchange: need a completed round and plane 0 or 1");
  if (e->begun) return fail(e, P2PG_ERR_STATE, "exchange: the next round has begun");
  if (plane == 1 && e->cfg.mode != P2PG_MODE_GOSSIP)
    return fail(e, P2PG_ERR_ARG, "exchange: plane 1 is for gossip pushes");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  const int r = e->round - 1;  // the round step() completed
  // plane 0 moves frontier rows owner -> ghost; plane 1 moves pushed rows ghost -> owner
  const bool use_send_list = (plane == 0) == pack;
  const int32_t* ids = use_send_list ? e->d_send : e->d_recv;
  const int64_t n = use_send_list ? e->n_send : e->n_recv;
  hipError_t rr = pack ? launch_pack(e->st, plane, r, ids, n, (uint64_t*)buf, e->stream)
                       : launch_unpack(e->st, plane, r, ids, n, (const uint64_t*)buf, e->stream);
  if (rr == hipSuccess) rr = hipStreamSynchronize(e->stream);
  if (rr != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("exchange: ") + hipGetErrorString(rr));
  return P2PG_OK;
}

int p2pg_exchange_pack(p2pg_engine* e, int32_t plane, void* dev_buf) {
  return exchange(e, plane, true, dev_buf);
}

int p2pg_exchange_unpack(p2pg_engine* e, int32_t plane, const void* dev_buf) {
  return exchange(e, plane, false, const_cast<void*>(dev_buf));
}

int p2pg_update_edges(p2pg_engine* e, int64_t n_add, const int32_t* add, int64_t n_del,
                      const int32_t* del) {
  if (!e || !e->d_rowptr || n_add < 0 || n_del < 0 || (n_add && !add) || (n_del && !del))
    return fail(e, P2PG_ERR_ARG, "update_edges: bad arguments");
  if (e->d_gid || (e->cfg.flags & P2PG_FLAG_LOCAL_GRAPH))
    return fail(e, P2PG_ERR_STATE, "update_edges: not supported on a vertex-partitioned rank");
  if (e->arr_round >= 0 && e->arr_round == e->round)
    return fail(e, P2PG_ERR_STATE, "update_edges: one update per round boundary");
  if (e->begun) return fail(e, P2PG_ERR_STATE, "update_edges: a round has begun (step_begin)");
  const int64_t V = e->V;
  const std::vector<int64_t>& rp = e->h_rowptr;
  const std::vector<int32_t>& ci = e->h_colidx;
  auto slot_of = [&](int32_t a, int32_t b) -> int64_t {  // slot of b in a's row, or -1
    const int32_t* beg = ci.data() + rp[a];
    const int32_t* end = ci.data() + rp[a + 1];
    const int32_t* it = std::lower_bound(beg, end, b);
    return (it != end && *it == b) ? (int64_t)(it - ci.data()) : -1;
  };
  // both directions of every change, sorted by (row, neighbour)
  std::vector<std::pair<int32_t, int32_t>> adds, dels;
  auto collect = [&](int64_t n, const int32_t* pr, bool is_add,
                     std::vector<std::pair<int32_t, int32_t>>& out) -> int {
    for (int64_t i = 0; i < n; ++i) {
      const int32_t a = pr[2 * i], b = pr[2 * i + 1];
      if (a < 0 || b < 0 || a >= V || b >= V)
        return fail(e, P2PG_ERR_ARG, "update_edges: peer id out of range");
      if (a == b)  // node.py:131-133 refuses self connections
        return fail(e, P2PG_ERR_ARG, "update_edges: self connection");
      const bool exists = slot_of(a, b) >= 0;
      if (is_add && exists)  // node.py:136-139: already connected
        return fail(e, P2PG_ERR_ARG, "update_edges: connection already exists");
      if (!is_add && !exists)  // node.py:178-189: not connected
        return fail(e, P2PG_ERR_ARG, "update_edges: no such connection");
      out.emplace_back(a, b);
      out.emplace_back(b, a);
    }
    std::sort(out.begin(), out.end());
    if (std::adjacent_find(out.begin(), out.end()) != out.end())
      return fail(e, P2PG_ERR_ARG, "update_edges: a connection is listed twice");
    return P2PG_OK;
  };
  int rc;
  if ((rc = collect(n_add, add, true, adds))) return rc;
  if ((rc = collect(n_del, del, false, dels))) return rc;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  // new adjacency: each row = old row - removed + added, ascending
  std::vector<int64_t> nrp(V + 1, 0);
  std::vector<int32_t> nci;
  nci.reserve(ci.size() + adds.size());
  {
    size_t ia = 0, id = 0;
    for (int64_t v = 0; v < V; ++v) {
      std::vector<int32_t> plus;
      while (ia < adds.size() && adds[ia].first == v) plus.push_back(adds[ia++].second);
      size_t k = 0;
      for (int64_t j = rp[v]; j < rp[v + 1]; ++j) {
        const int32_t u = ci[j];
        if (id < dels.size() && dels[id].first == v && dels[id].second == u) {
          ++id;
          continue;
        }
        while (k < plus.size() && plus[k] < u) nci.push_back(plus[k++]);
        nci.push_back(u);
      }
      while (k < plus.size()) nci.push_back(plus[k++]);
      nrp[v + 1] = (int64_t)nci.size();
    }
  }
  const bool running = e->have_state && e->round > 0 && !e->done;
  if (running) {
    // Messages sent in the last round are in flight on the OLD connections: the ones on removed
    // connections are lost (a stopped NodeConnection drops its unread buffer,
    // nodeconnection.py:192-228), the rest arrive next round.  Materialize them as row pushes
    // next[round&1] over the old graph minus the removed slots, before the graph changes.
    DevState& s = e->st;
    const bool gossip = e->cfg.mode == P2PG_MODE_GOSSIP;
    std::vector<uint8_t> gone(ci.size(), 0);
    for (const auto& d : dels) gone[slot_of(d.first, d.second)] = 1;
    uint8_t* d_gone = nullptr;
    HIPCHK(e, hipMalloc((void**)&d_gone, gone.empty() ? 1 : gone.size()));
    if (!gone.empty()) HIPCHK(e, hipMemcpy(d_gone, gone.data(), gone.size(), hipMemcpyHostToDevice));
    if (!dels.empty()) {
      // the arrivals of the next round lose the sends in flight on the removed connections: count
      // the last round's lost sends again with those slots gone (churn losses included), while the
      // graph its own arrivals travelled on (the senders' first receipts) is still at hand
      DevGraph gs = graph(e);
      gs.gone = d_gone;
      hipError_t x = enqueue_lost_count(e, gs, graph_for_arrivals(e, e->round - 1), e->round - 1);
      if (x == hipSuccess) x = hipStreamSynchronize(e->stream);
      if (x != hipSuccess) {
        (void)hipFree(d_gone);
        return fail(e, P2PG_ERR_HIP, std::string("update_edges (lost sends): ") + hipGetErrorString(x));
      }
      e->lost_last = (uint64_t)e->h_cnt2[1];
    }
    free_arr(e);
    e->d_gone = d_gone;
    if (!s.next[0]) {  // flood: row-push planes on first use
      for (int i = 0; i < 2; ++i) {
        HIPCHK(e, hipMalloc((void**)&s.next[i], e->plane_bytes ? e->plane_bytes : 8));
        HIPCHK(e, hipMalloc((void**)&s.T[i], e->bm_bytes ? e->bm_bytes : 8));
        HIPCHK(e, hipMemsetAsync(s.next[i], 0, e->plane_bytes, e->stream));
        HIPCHK(e, hipMemsetAsync(s.T[i], 0, e->bm_bytes, e->stream));
      }
    }
    DevGraph gold = graph(e);
    gold.gone = e->d_gone;
    RoundParams p = params(e);
    const int nx = e->round & 1;
    hipError_t lr;
    if (!gossip) {
      if (!e->consume_next) {
        lr = launch_materialize(gold, s, p, true, e->stream);
        if (lr != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("update_edges: ") + hipGetErrorString(lr));
      }
    } else {
      // the pushes of the last round, recomputed (Philox picks are a pure function of the
      // round, peer and message) as row atomics over the old graph without the removed slots
      HIPCHK(e, hipMemsetAsync(s.next[nx], 0, e->plane_bytes, e->stream));
      HIPCHK(e, hipMemsetAsync(s.T[nx], 0, e->bm_bytes, e->stream));
      p.round = e->round - 1;
      lr = launch_scatter_atomic(e, gold, p, e->prev_aw);
      if (lr != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("update_edges: ") + hipGetErrorString(lr));
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->wlist_check) {
      unsigned long long listed = 0;
      HIPCHK(e, hipMemcpy(&listed, s.stats + STAT_COUNT, sizeof(listed), hipMemcpyDeviceToHost));
      if (int rc2 = check_scatter_list(e, listed)) return rc2;
    }
    e->consume_next = true;
    e->last_push_e = false;
    e->stats_clear = true;  // the re-push above counted into the round counters
    // keep the old rows for the parents of the receiving round (record / deliveries)
    e->d_rowptr_arr = e->d_rowptr;
    e->d_colidx_arr = e->d_colidx;
    e->d_rowptr = nullptr;
    e->d_colidx = nullptr;
    e->arr_round = e->round;
  }
  std::vector<uint32_t> rev;
  if ((rc = check_csr(e, V, nrp.data(), nci.data(), rev))) return rc;
  if ((rc = upload_graph(e, V, nrp.data(), nci.data(), rev))) return rc;
  if (e->have_state && (rc = alloc_edge_planes(e))) return rc;
  return P2PG_OK;
}

}  // extern "C"

namespace {

constexpr uint64_t SNAP_MAGIC = 0x50414E5347503250ull;  // "P2PGSNAP"
constexpr uint32_t SNAP_VERSION = 3;  // 2: + last_new; 3: + sent_last / lost_last

struct SnapHeader {
  uint64_t magic;
  uint32_t version, mode;
  int64_t V, nnz;
  int32_t M, W, fanout, round;
  uint32_t flags, churn_threshold, msg_id_base, done;
  uint32_t consume_next, has_next;
  uint64_t gossip_seed, churn_seed, graph_hash, src_hash, total_relays, prev_aw, prev_av;
  uint64_t last_new;  // first receipts of the last round (deliveries, decay-phase push dedup)
  uint64_t sent_last, lost_last;  // the next round's arrivals (p2pg_round_stats.received)
};

uint64_t fnv1a(uint64_t h, const void* data, size_t n) {
  const unsigned char* p = (const unsigned char*)data;
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= 0x100000001B3ull;
  }
  return h;
}

uint64_t graph_hash(const p2pg_engine* e) {
  uint64_t h = fnv1a(0xCBF29CE484222325ull, e->h_rowptr.data(), e->h_rowptr.size() * sizeof(int64_t));
  return fnv1a(h, e->h_colidx.data(), e->h_colidx.size() * sizeof(int32_t));
}

int64_t snapshot_bytes(const p2pg_engine* e, bool with_next, bool with_record) {
  int64_t n = (int64_t)sizeof(SnapHeader) + 2 * (int64_t)e->plane_bytes + 2 * (int64_t)e->bm_bytes;
  if (with_next) n += (int64_t)e->plane_bytes + (int64_t)e->bm_bytes;
  if (with_record) n += 2 * (int64_t)e->V * e->M * (int64_t)sizeof(int32_t);
  return n;
}

int64_t snapshot_bytes(const p2pg_engine* e) {
  return snapshot_bytes(e, e->st.next[0] != nullptr, e->st.hop != nullptr);
}

// The planes of a snapshot, in order: seen, saturated bits, the last round's activity bits and
// frontier (its first receipts), [pending row pushes + their bits], [hop, parent].
template <class F>
int for_planes(p2pg_engine* e, bool with_next, F&& f) {
  DevState& s = e->st;
  const int last = (e->round + 1) & 1;  // (round - 1) & 1
  const int nx = e->round & 1;
  int rc;
  if ((rc = f((void*)s.seen, e->plane_bytes))) return rc;
  if ((rc = f((void*)s.S, e->bm_bytes))) return rc;
  if ((rc = f((void*)s.A[last], e->bm_bytes))) return rc;
  if ((rc = f((void*)s.F[last], e->plane_bytes))) return rc;
  if (with_next) {
    if ((rc = f((void*)s.next[nx], e->plane_bytes))) return rc;
    if ((rc = f((void*)s.T[nx], e->bm_bytes))) return rc;
  }
  if (s.hop) {
    const size_t hb = (size_t)e->V * e->M * sizeof(int32_t);
    if ((rc = f((void*)s.hop, hb))) return rc;
    if ((rc = f((void*)s.parent, hb))) return rc;
  }
  return P2PG_OK;
}

}  // namespace

extern "C" {

int p2pg_snapshot_size(p2pg_engine* e, int64_t* bytes) {
  if (!e || !bytes) return fail(e, P2PG_ERR_ARG, "snapshot_size: bad arguments");
  if (!e->have_state) return fail(e, P2PG_ERR_STATE, "snapshot_size: no sources set");
  *bytes = snapshot_bytes(e);
  return P2PG_OK;
}

int p2pg_snapshot(p2pg_engine* e, void* buf, int64_t cap) {
  if (!e || !buf) return fail(e, P2PG_ERR_ARG, "snapshot: bad arguments");
  if (!e->have_state) return fail(e, P2PG_ERR_STATE, "snapshot: no sources set");
  if (e->begun) return fail(e, P2PG_ERR_STATE, "snapshot: a round has begun (step_begin)");
  if (e->arr_round >= 0 && e->arr_round == e->round)
    return fail(e, P2PG_ERR_STATE, "snapshot: take it before a topology update or after the next round");
  if (!e->frontier_kept)
    return fail(e, P2PG_ERR_STATE, "snapshot: the last round's frontier was not kept");
  if (e->d_gid && e->cfg.mode == P2PG_MODE_GOSSIP && e->last_push_e && e->round > 0 && !e->done)
    return fail(e, P2PG_ERR_STATE,
                "snapshot: a partitioned rank holds this round's pushes per connection; take it "
                "after a sparse round");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  DevState& s = e->st;
  if (e->cfg.mode == P2PG_MODE_GOSSIP && e->last_push_e && e->round > 0 && !e->done) {
    // pushes held per connection (E) -> row pushes, so the state does not depend on slots
    RoundParams p = params(e);
    hipError_t lr = launch_materialize(graph(e), s, p, false, e->stream);
    if (lr != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("snapshot: ") + hipGetErrorString(lr));
    e->last_push_e = false;
    e->stats_clear = true;
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  const int64_t need = snapshot_bytes(e);
  if (cap < need) return fail(e, P2PG_ERR_ARG, "snapshot: buffer smaller than p2pg_snapshot_size");
  SnapHeader h{};
  h.magic = SNAP_MAGIC;
  h.version = SNAP_VERSION;
  h.mode = (uint32_t)e->cfg.mode;
  h.V = e->V;
  h.nnz = e->nnz;
  h.M = e->M;
  h.W = e->W;
  h.fanout = e->cfg.fanout;
  h.round = e->round;
  h.flags = e->cfg.flags & P2PG_FLAG_RECORD;
  h.churn_threshold = e->cfg.churn_threshold;
  h.msg_id_base = e->cfg.msg_id_base;
  h.done = e->done ? 1u : 0u;
  h.consume_next = e->consume_next ? 1u : 0u;
  h.has_next = s.next[0] ? 1u : 0u;
  h.gossip_seed = e->cfg.gossip_seed;
  h.churn_seed = e->cfg.churn_seed;
  h.graph_hash = graph_hash(e);
  h.src_hash = fnv1a(0xCBF29CE484222325ull, e->h_src.data(), e->h_src.size() * sizeof(int32_t));
  h.total_relays = e->total_relays;
  h.prev_aw = e->prev_aw;
  h.prev_av = e->prev_av;
  h.last_new = e->last_new;
  h.sent_last = e->sent_last;
  h.lost_last = e->lost_last;
  char* out = (char*)buf;
  std::memcpy(out, &h, sizeof(h));
  size_t off = sizeof(h);
  return for_planes(e, s.next[0] != nullptr, [&](void* dev, size_t n) -> int {
    if (n) HIPCHK(e, hipMemcpy(out + off, dev, n, hipMemcpyDeviceToHost));
    off += n;
    return P2PG_OK;
  });
}

int p2pg_restore(p2pg_engine* e, const void* buf, int64_t size) {
  if (!e || !buf || size < (int64_t)sizeof(SnapHeader)) return fail(e, P2PG_ERR_ARG, "restore: bad arguments");
  if (!e->have_state) return fail(e, P2PG_ERR_STATE, "restore: set the same sources first");
  if (e->begun) return fail(e, P2PG_ERR_STATE, "restore: a round has begun (step_begin)");
  SnapHeader h;
  std::memcpy(&h, buf, sizeof(h));
  if (h.magic != SNAP_MAGIC || h.version != SNAP_VERSION)
    return fail(e, P2PG_ERR_ARG, "restore: not a relay-engine snapshot");
  if (h.mode != (uint32_t)e->cfg.mode || h.fanout != e->cfg.fanout ||
      h.gossip_seed != e->cfg.gossip_seed || h.churn_seed != e->cfg.churn_seed ||
      h.churn_threshold != e->cfg.churn_threshold || h.msg_id_base != e->cfg.msg_id_base ||
      h.flags != (e->cfg.flags & P2PG_FLAG_RECORD))
    return fail(e, P2PG_ERR_STATE, "restore: engine configuration differs from the snapshot's");
  if (h.V != e->V || h.nnz != e->nnz || h.graph_hash != graph_hash(e))
    return fail(e, P2PG_ERR_STATE, "restore: graph differs from the snapshot's");
  if (h.M != e->M || h.src_hash != fnv1a(0xCBF29CE484222325ull, e->h_src.data(), e->h_src.size() * sizeof(int32_t)))
    return fail(e, P2PG_ERR_STATE, "restore: broadcast sources differ from the snapshot's");
  // validate everything before the engine is touched: a rejected snapshot leaves it as it was
  if (h.round < 0 || h.has_next > 1 || h.done > 1 || h.consume_next > 1 ||
      (h.consume_next && !h.has_next))
    return fail(e, P2PG_ERR_ARG, "restore: corrupt snapshot header");
  const bool with_next = h.has_next != 0;
  if (size < snapshot_bytes(e, with_next, (h.flags & P2PG_FLAG_RECORD) != 0))
    return fail(e, P2PG_ERR_ARG, "restore: snapshot truncated");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  DevState& s = e->st;
  if (with_next && !s.next[0]) {  // flood run that had a topology update
    for (int i = 0; i < 2; ++i) {
      HIPCHK(e, hipMalloc((void**)&s.next[i], e->plane_bytes ? e->plane_bytes : 8));
      HIPCHK(e, hipMalloc((void**)&s.T[i], e->bm_bytes ? e->bm_bytes : 8));
    }
  }
  int rc = p2pg_reset(e);
  if (rc) return rc;
  if (s.next[0]) {  // pending pushes: from the snapshot, or none (a flood snapshot without them)
    for (int i = 0; i < 2; ++i) {
      HIPCHK(e, hipMemsetAsync(s.next[i], 0, e->plane_bytes, e->stream));
      HIPCHK(e, hipMemsetAsync(s.T[i], 0, e->bm_bytes, e->stream));
    }
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  e->round = h.round;
  e->done = h.done != 0;
  e->consume_next = h.consume_next != 0;
  e->last_push_e = false;
  e->total_relays = h.total_relays;
  e->prev_aw = h.prev_aw;
  e->prev_av = h.prev_av;
  e->last_new = h.last_new;
  e->sent_last = h.sent_last;
  e->lost_last = h.lost_last;
  // the snapshot holds the last round's frontier, not the one before it, so that round's
  // delivery parents cannot be found (round 0's are -1): deliveries refuse it, as documented
  e->frontier_kept = true;
  e->frontier_kept_prev = h.round <= 1;
  e->prev2_aw = e->prev2_av = e->prev2_new = 0;  // no growth history: no update+push prediction
  const char* in = (const char*)buf;
  size_t off = sizeof(h);
  rc = for_planes(e, with_next, [&](void* dev, size_t n) -> int {
    if (n) HIPCHK(e, hipMemcpy(dev, in + off, n, hipMemcpyHostToDevice));
    off += n;
    return P2PG_OK;
  });
  if (rc) return rc;
  HIPCHK(e, hipMemsetAsync(s.A[e->round & 1], 0, e->bm_bytes, e->stream));
  // the last round's active-word masks are not in the snapshot: rebuilt from its frontier rows
  // (a re-push after a topology update, and the next sparse push, list words by them)
  if (e->round > 0) {
    hipError_t x = launch_rebuild_aw(s, e->round - 1, e->V, e->stream);
    if (x == hipSuccess) x = hipStreamSynchronize(e->stream);
    if (x != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("restore: ") + hipGetErrorString(x));
  }
  return P2PG_OK;
}

int p2pg_kernel_times(p2pg_engine* e, double ms[P2PG_KCLASS_N], int64_t launches[P2PG_KCLASS_N]) {
  if (!e) return P2PG_ERR_ARG;
  if (!e->ev_cls.empty()) {
    // launches still unresolved: a run whose last rounds went without a counter read-back (a
    // batched flood or decay tail) -- wait for them, so the sums cover every launch counted
    HIPCHK(e, hipSetDevice(e->cfg.device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const int r = resolve_timings(e);
    if (r) return r;
  }
  for (int i = 0; i < P2PG_KCLASS_N; ++i) {
    if (ms) ms[i] = e->kms[i];
    if (launches) launches[i] = e->klaunch[i];
  }
  return P2PG_OK;
}

int p2pg_set_timed_classes(p2pg_engine* e, uint32_t mask) {
  if (!e) return P2PG_ERR_ARG;
  if (mask >> P2PG_KCLASS_N) return fail(e, P2PG_ERR_ARG, "set_timed_classes: unknown class bit");
  e->timed_mask = mask;
  return P2PG_OK;
}

int p2pg_device_philox(p2pg_engine* e, int32_t n, const uint32_t* ctr, const uint32_t key[2],
                       uint32_t* out) {
  if (!e || n < 0 || (n > 0 && (!ctr || !key || !out))) return fail(e, P2PG_ERR_ARG, "device_philox: bad arguments");
  if (n == 0) return P2PG_OK;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  uint32_t *dc = nullptr, *dout = nullptr;
  HIPCHK(e, hipMalloc((void**)&dc, sizeof(uint32_t) * 4 * n));
  HIPCHK(e, hipMalloc((void**)&dout, sizeof(uint32_t) * 4 * n));
  hipError_t r = hipMemcpy(dc, ctr, sizeof(uint32_t) * 4 * n, hipMemcpyHostToDevice);
  if (r == hipSuccess) r = launch_philox(n, dc, key[0], key[1], dout, e->stream);
  if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
  if (r == hipSuccess) r = hipMemcpy(out, dout, sizeof(uint32_t) * 4 * n, hipMemcpyDeviceToHost);
  (void)hipFree(dc);
  (void)hipFree(dout);
  if (r != hipSuccess) return fail(e, P2PG_ERR_HIP, std::string("device_philox: ") + hipGetErrorString(r));
  return P2PG_OK;
}

const char* p2pg_last_error(const p2pg_engine* e) { return e ? e->err.c_str() : p2pg_global_error(); }

void p2pg_destroy(p2pg_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->cfg.device);
  (void)hipStreamSynchronize(e->stream);
  free_state(e);
  free_graph(e);
  if (e->h_stats) (void)hipHostFree(e->h_stats);
  if (e->h_bstats) (void)hipHostFree(e->h_bstats);
  if (e->d_bstats) (void)hipFree(e->d_bstats);
  for (int i = 0; i < 2; ++i)
    if (e->ev[i]) (void)hipEventDestroy(e->ev[i]);
  for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
  if (e->ev_sync) (void)hipEventDestroy(e->ev_sync);
  if (e->ev_spare) (void)hipEventDestroy(e->ev_spare);
  if (e->ev_main) (void)hipEventDestroy(e->ev_main);
  if (e->side) (void)hipStreamDestroy(e->side);
  if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
  delete e;
}

}  // extern "C"
