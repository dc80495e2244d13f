// Gossip sparse rounds: the row-atomic push of a round's first receipts, lane-parallel.
//
// Why: in a sparse round (few active words per active peer: config 4's rounds 0-8 and 26-45
// carry 1-2 new bits per active peer) the per-source scatter of relay_kernels.hip
// (k_gossip_scatter<.., false>: one wave per source, lane = word, LDS mask table, flush per
// neighbour chunk) spends a whole wave visit -- compaction scan, table clear, one pick batch,
// flush loop -- on one or two bits.  Here the three levels of a push are flattened onto lanes:
//   level 1  lane = active peer u     (64 tasks of the A bitmap per wave pass, compacted):
//            the active-word mask AW[u] (W <= 8: the nonzero words of the row);
//   level 2  its (u, w) pairs are listed in peer order (k_sparse_words, two passes) ...
//   level 3  ... which k_sparse_push hands out 64 words per wave pass (a hub's words spread over
//            many waves; one wave per 64 peers left the hub tasks' wave 10x behind), lane =
//            (u, w, bit b): Philox + Floyd picks of message w*64+b (gossip_picks_t),
//            then, per distinct (u, w, target): one atomicOr of the merged mask into
//            next[target][w] and a byte store into the target's touched byte (the same pushes,
//            and the same count of distinct (sender, target, word) masks, as the per-source
//            kernel); k_touched_bits folds the bytes into the T bitmap.
// Each level's entries are handed out 64 at a time; the owner lane of an entry is found by a
// marker + running-max scan and its index inside the owner by select-nth-bit, so no per-bit
// loop runs on one lane.  Level-3 passes never split a word's bits (at most 64), so a mask is
// merged and counted once.  Reference semantics: Node.send_to_nodes -> send_to_node per chosen
// connection (node.py:106-120), counted before sending; lost sends (churn, a connection removed
// by a topology update) push nothing (nodeconnection.py:123-126).
#include "device_util.h"

namespace p2pg {
namespace {

template <int KP>
struct SparseLds {
  uint32_t own[64];     // owner markers of the current pass
  uint32_t bit[64];     // level-3 entry -> its message bit
  uint32_t pk[KP][64];  // level-3 entry -> its picks (slot offsets in the sender's row)
};

// Owner lane of entry pb + lane of a pass over per-lane ranges [pos, pos + cnt) (pos is the
// exclusive prefix sum of cnt): every range that meets the pass marks its first slot, and a
// running maximum fills the rest.  Whole wave active.
__device__ __forceinline__ int pass_owner(uint32_t* own, int lane, uint32_t pos, uint32_t cnt,
                                          uint32_t pb) {
  own[lane] = 0u;
  wave_lds_sync();
  if (cnt && pos + cnt > pb && pos < pb + 64u) own[pos > pb ? pos - pb : 0u] = (uint32_t)lane;
  wave_lds_sync();
  return (int)wave_scan_max_u32(own[lane]);
}

// Levels 1-2: the (active peer, active word) pairs of round r's frontier, listed as u << 6 | w
// in peer order, without atomics: pass COUNT counts each chunk's pairs (SW_TASKS task words per
// chunk), k_chunk_scan turns the counts into offsets, pass WRITE stores the pairs there, 64 per
// store instruction (lane = pair: owner peer by pass_owner, word by select-nth-bit).  A single
// list counter took one same-address atomic per 64 peers: ~8 ns each, serialized (0.1-1.2 ms
// per round).  Chunks are small because the Barabasi-Albert hubs (lowest ids, most active
// words) share the first tasks.
#ifndef P2PG_SW_TASKS
#define P2PG_SW_TASKS 16
#endif
constexpr int SW_TASKS = P2PG_SW_TASKS;
#ifndef P2PG_SPARSE_GRID_MAX
#define P2PG_SPARSE_GRID_MAX 8192
#endif
constexpr int64_t SPARSE_GRID_MAX = P2PG_SPARSE_GRID_MAX;

template <bool WRITE>
__global__ __launch_bounds__(256) void k_sparse_words(DevGraph g, DevState st, RoundParams p,
                                                      SparseBufs b) {
  __shared__ uint32_t own_all[WPB][64];
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  uint32_t* own = own_all[wib];
  const int64_t V = g.V;
  const int W = st.W;
  const int cur = p.round & 1;
  const uint64_t* __restrict__ Fc = st.F[cur];
  const uint64_t* __restrict__ AWc = st.AW[cur];
  const uint32_t* __restrict__ Ac = st.A[cur];
  const int64_t ntasks = (V + 31) >> 5;
  for (int64_t tb = ((int64_t)blockIdx.x * WPB + wib) * SW_TASKS; tb < ntasks;
       tb += (int64_t)gridDim.x * WPB * SW_TASKS) {
    const int64_t chunk = tb / SW_TASKS;
    const int64_t tl = tb + lane;
    const uint32_t al = lane < SW_TASKS && tl < ntasks ? Ac[tl] : 0u;
    if (!__ballot(al != 0u)) {
      if (!WRITE && lane == 0) b.chunk_cnt[chunk] = 0u;
      continue;
    }
    const uint32_t pc = (uint32_t)__popc(al);
    const uint32_t pinc = wave_scan_u32(pc);
    const uint32_t pos = pinc - pc;
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)pinc, 63);
    uint64_t base = WRITE ? b.chunk_off[chunk] : 0ull;  // wave-uniform
    uint32_t nwords = 0;
    for (uint32_t pb = 0; pb < total; pb += 64) {
      // lane = active peer pb + lane of this chunk
      const int ow = pass_owner(own, lane, pos, pc, pb);
      const uint32_t opos = bperm(ow, pos), oal = bperm(ow, al);
      int64_t u = 0;
      uint64_t am = 0;
      if (pb + (uint32_t)lane < total) {
        u = ((tb + ow) << 5) + select_bit32(oal, pb + (uint32_t)lane - opos);
        if (AWc) {
          am = AWc[u];
        } else {  // W <= PACK_W_MAX_PLAIN: the nonzero words of the row
          for (int w = 0; w < W; ++w) am |= (uint64_t)(at_row(Fc, u, W)[w] != 0ull) << w;
        }
      }
      const uint32_t wc = (uint32_t)__popcll(am);
      const uint32_t winc = wave_scan_u32(wc);
      const uint32_t wpos = winc - wc;
      const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)winc, 63);
      nwords += wtot;
      if (WRITE) {
        // lane = pair wb + lane of these peers
        for (uint32_t wb = 0; wb < wtot; wb += 64) {
          const int pw = pass_owner(own, lane, wpos, wc, wb);
          const uint32_t ppos = bperm(pw, wpos);
          const uint64_t pam = bperm64(pw, am);
          const uint64_t pu = bperm64(pw, (uint64_t)u);
          const uint64_t idx = base + wb + (uint64_t)lane;
          if (wb + (uint32_t)lane < wtot && idx < (uint64_t)b.cap)
            b.list[idx] = (pu << 6) | select_bit64(pam, wb + (uint32_t)lane - ppos);
        }
        base += wtot;
      }
    }
    if (!WRITE && lane == 0) b.chunk_cnt[chunk] = nwords;
  }
}

// Exclusive prefix sum of the chunk counts (one block): chunk_off, and the total into *count.
// Tiles of 16 waves x 64 lanes x CPT counts; wave v scans its contiguous 64 * CPT counts as CPT
// rows of 64 (lane = count: 16 B-per-lane loads and 8 B-per-lane stores, every row one 256 B /
// 512 B contiguous access), then the 16 wave totals offset the waves.  One tile covers config
// 4's 19.5K chunks.  (Thread-major runs -- CPT consecutive counts per thread -- left every store
// instruction 64 partial lines apart: 13 us per launch, a fixed cost of every sparse round.)
// Row sums within a wave's segment stay 32-bit: <= 64 * CPT chunks x SW_TASKS * 32 peers x 64
// words < 2^32.
constexpr int CPT = 24;
static_assert((uint64_t)64 * CPT * SW_TASKS * 32 * 64 < (1ull << 32), "32-bit segment sums");
__global__ __launch_bounds__(1024) void k_chunk_scan(int64_t n, SparseBufs b) {
  __shared__ uint64_t wsum[16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint64_t carry = 0;
  for (int64_t tile = 0; tile < n; tile += 16 * 64 * CPT) {
    const int64_t s0 = tile + (int64_t)wv * 64 * CPT + lane;
    uint32_t c[CPT];
#pragma unroll
    for (int j = 0; j < CPT; ++j) {  // all loads first
      const int64_t i = s0 + 64 * j;
      c[j] = i < n ? b.chunk_cnt[i] : 0u;
    }
    uint32_t x[CPT];  // exclusive offsets within the wave's segment
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const uint32_t inc = wave_scan_u32(c[j]);
      x[j] = run + inc - c[j];
      run += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    }
    if (lane == 0) wsum[wv] = run;
    __syncthreads();
    uint64_t before = carry, all = carry;
    for (int i = 0; i < 16; ++i) {
      if (i < wv) before += wsum[i];
      all += wsum[i];
    }
    __syncthreads();  // wsum is rewritten by the next tile
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int64_t i = s0 + 64 * j;
      if (i < n) b.chunk_off[i] = before + x[j];
    }
    carry = all;
  }
  if (t == 0) *b.count = (unsigned long long)carry;
}

// Level 3: lane = (peer, word, bit) of the listed words, 64 words per wave pass (balanced: a
// hub's words spread over many waves).  A bit pass [b0, b1) holds whole words only.
template <bool CHURN, int K>
__global__ __launch_bounds__(256) void k_sparse_push(DevGraph g, DevState st, RoundParams p,
                                                     SparseBufs sb) {
  constexpr int KP = K > 0 ? K : 16;
  __shared__ SparseLds<KP> lds[WPB];
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  SparseLds<KP>& L = lds[wib];
  const int W = st.W;
  const int cur = p.round & 1, nxt = cur ^ 1;
  const uint64_t* __restrict__ Fc = st.F[cur];
  uint64_t* __restrict__ nx = st.next[nxt];
  const uint32_t k = K > 0 ? (uint32_t)K : (uint32_t)p.fanout;
  const uint64_t* __restrict__ list = sb.list;
  uint8_t* __restrict__ touched = sb.touched;
  const int64_t listed = (int64_t)ldc(sb.count);
  const int64_t n = listed < sb.cap ? listed : sb.cap;
  uint64_t pushed = 0;  // distinct (sender, target, word) masks pushed by this lane

  for (int64_t e0 = ((int64_t)blockIdx.x * WPB + wib) * 64; e0 < n;
       e0 += (int64_t)gridDim.x * WPB * 64) {
    uint32_t w = 0, deg = 0;
    int64_t u = 0, rb = 0;
    uint64_t f = 0;
    if (e0 + lane < n) {
      const uint64_t x = list[e0 + lane];
      u = (int64_t)(x >> 6);
      w = (uint32_t)(x & 63u);
      rb = g.rowptr[u];
      deg = (uint32_t)(g.rowptr[u + 1] - rb);
      f = at_row(Fc, u, W)[w];
    }
    const uint32_t bc = (uint32_t)__popcll(f);
    const uint32_t binc = wave_scan_u32(bc);
    const uint32_t bpos = binc - bc;
    const uint32_t btot = (uint32_t)__builtin_amdgcn_readlane((int)binc, 63);
    for (uint32_t b0 = 0; b0 < btot;) {
      const uint64_t over = __ballot(bc != 0u && bpos >= b0 && bpos + bc > b0 + 64u);
      const uint32_t b1 =
          over ? (uint32_t)__builtin_amdgcn_readlane((int)bpos, (int)__builtin_ctzll(over)) : btot;
      const int bw = pass_owner(L.own, lane, bpos, bc, b0);
      const uint32_t gpos = bperm(bw, bpos), gcnt = bperm(bw, bc);
      const uint64_t gf = bperm64(bw, f);
      const uint32_t gw = bperm(bw, w), gdeg = bperm(bw, deg);
      const int64_t gu = (int64_t)bperm64(bw, (uint64_t)u);
      const int64_t grb = (int64_t)bperm64(bw, (uint64_t)rb);
      const bool bv = (uint32_t)lane < b1 - b0;
      const uint32_t gs = gpos - b0, ge = gs + gcnt;  // this word's entries [gs, ge)
      uint32_t b = 0, gv = 0;
      if (bv) {
        b = select_bit64(gf, b0 + (uint32_t)lane - gpos);
        gv = gidx(g, gu);
        L.bit[lane] = b;
        if (gdeg > k) {
          const uint32_t mg = p.msg_base + gw * 64u + b;
          if constexpr (K > 0) {
            uint32_t pk[K];
            gossip_picks_t<K>((uint32_t)p.round, gv, mg, gdeg, p.gseed_lo, p.gseed_hi, pk);
#pragma unroll
            for (int q = 0; q < K; ++q) L.pk[q][lane] = pk[q];
          } else {
            uint32_t pk[16];
            gossip_picks((uint32_t)p.round, gv, mg, gdeg, (int)k, p.gseed_lo, p.gseed_hi, pk);
            for (uint32_t q = 0; q < k; ++q) L.pk[q][lane] = pk[q];
          }
        }
      }
      wave_lds_sync();
      if (bv) {
        const bool all = gdeg <= k;  // every connection, the whole word at once
        const uint32_t kk = all ? gdeg : k;
        for (uint32_t q = 0; q < kk; ++q) {
          uint32_t t;
          uint64_t mask;
          if (all) {
            if ((uint32_t)lane != gs) break;
            t = q;
            mask = gf;
          } else {
            t = L.pk[q][lane];
            // first entry of this word to pick t?  Then it pushes the word's merged mask.
            bool lead = true;
            for (uint32_t i = gs; i < (uint32_t)lane && lead; ++i)
              for (uint32_t q2 = 0; q2 < k; ++q2) lead &= L.pk[q2][i] != t;
            if (!lead) continue;
            mask = 1ull << b;
            for (uint32_t i = (uint32_t)lane + 1u; i < ge; ++i) {
              bool hit = false;
              for (uint32_t q2 = 0; q2 < k; ++q2) hit |= L.pk[q2][i] == t;
              if (hit) mask |= 1ull << L.bit[i];
            }
          }
          const int64_t slot = grb + (int64_t)t;
          if (g.gone && g.gone[slot]) continue;  // connection removed: the push is lost
          const int32_t v = g.colidx[slot];
          if (CHURN && churn_dropped((uint32_t)p.round, gv, gidx(g, v), p.churn_thr, p.cseed_lo,
                                     p.cseed_hi))
            continue;
          pushed += 1;  // a distinct (sender, target, word) mask, counted before the dedup
          if (p.dedup_push) {
            mask &= ~at_row(st.seen, v, W)[gw];
            if (!mask) continue;  // a duplicate in its entirety: nothing to deliver
          }
          atomicOr((unsigned long long*)at_row(nx, v, W) + gw, (unsigned long long)mask);
          touched[v] = 1u;  // a plain byte store: a T-bitmap atomic here doubled the atomics
        }
      }
      wave_lds_sync();  // the entries' LDS is rewritten by the next pass
      b0 = b1;
    }
  }
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};
  c[ST_SCATTER] = pushed;
  flush_stats(st.stats, c, lane);
}

// The touched bytes of k_sparse_push -> T bits of round r+1 (one lane per 32-peer task word,
// the only writer of that word here), bytes cleared for the next sparse round.
__global__ __launch_bounds__(256) void k_touched_bits(int64_t V, uint32_t* __restrict__ T,
                                                      uint8_t* __restrict__ touched) {
  const int64_t ntasks = (V + 31) >> 5;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntasks;
       t += (int64_t)gridDim.x * blockDim.x) {
    uint4* q = reinterpret_cast<uint4*>(touched + (t << 5));  // V is padded to 32 peers
    const uint4 a = q[0], b = q[1];
    const uint32_t wv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) m |= ((wv[i] >> (8 * j)) & 1u) << (4 * i + j);
    if (m) {
      T[t] |= m;
      q[0] = make_uint4(0u, 0u, 0u, 0u);
      q[1] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Dense (E-form) push of the pull hubs (deg > HUB_T) in fused rounds.  The per-source scatter
// covers a wide source with one wave per 16-connection chunk, and every chunk wave recomputes
// ALL the source's picks (only those landing in its chunk are kept): ceil(deg / 16) x the
// Philox work, 625 x for a 10K-connection hub (c4: ~0.8 ms per early fused round for 764
// hubs).  Here the picks run once:
//   k_wide_zero: the receiver-slot E rows of every active hub are zeroed (its nf packed words,
//                or W words unpacked) -- receivers gather them whole;
//   k_wide_push: one wave per hub, lane = (word, bit): Philox + Floyd picks, then per pick one
//                atomicOr of the message bit into E[r&1][rev[slot]] at the word's packed
//                position; a pick that finds the word still zero counts one nonzero (sender,
//                target, word) mask.  Churn-dropped connections keep zero rows.
// Atomics suit hubs: they carry few bits per round (a hub receives each message once).  The
// same path for the first dense round's deg > GCHUNK sources (625K of them in c4) measured
// slower than their chunk items (zeroing 2.4 ms + picks 1.0 ms vs ~1.7 ms), and a (source,
// word) list with merged masks was 3x slower for hubs (many bits per word: long merge loops).
static_assert(GCHUNK >= 16, "wide sources must have deg > fanout (<= 16)");

// Metadata lane = (item 4i + lane / 16, slot lane % 16): 4 chunk items per wave pass, all their
// row offsets / word masks / receiver slots gathered at once; then one store instruction per
// receiver row, lane = word (coalesced: a lane-per-row store pattern scattered 8 B writes over
// 64 rows per instruction and took 16 ms in c4's first dense round)
__global__ __launch_bounds__(256) void k_wide_zero(DevGraph g, DevState st, RoundParams p,
                                                   const int64_t* __restrict__ items,
                                                   int64_t n_items) {
  const int lane = threadIdx.x & 63;
  const int W = st.W;
  const int cur = p.round & 1;
  uint64_t* __restrict__ Eo = st.E[cur];
  const uint64_t* __restrict__ AWc = st.AW[cur];
  for (int64_t i0 = ((int64_t)blockIdx.x * WPB + wave_in_block()) * 4; i0 < n_items;
       i0 += (int64_t)gridDim.x * WPB * 4) {
    const int64_t it = i0 + (lane >> 4);
    const int s = lane & 15;
    int nf = 0;
    uint32_t row = 0;
    if (it < n_items) {
      const int64_t item = items[it];
      const int64_t v = item >> 32;
      if (bit_test(st.A[cur], v)) {
        const int64_t rb = g.rowptr[v], deg = g.rowptr[v + 1] - rb;
        const int64_t nb = (item & 0xFFFFFFFFll) * GCHUNK;
        if (nb + s < deg) {
          row = g.rev[rb + nb + s];
          nf = AWc ? __popcll(AWc[v]) : W;
        }
      }
    }
    for (uint64_t m = __ballot(nf > 0); m; m &= m - 1ull) {
      const int l = __builtin_ctzll(m);
      const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)row, l);
      const int n = __builtin_amdgcn_readlane(nf, l);
      if (lane < n) st_row(&Eo[(int64_t)r * W + lane], 0ull);
    }
  }
}

template <bool CHURN, int K>
__global__ __launch_bounds__(256) void k_wide_push(DevGraph g, DevState st, RoundParams p,
                                                   const int32_t* __restrict__ wide,
                                                   int64_t n_wide) {
  __shared__ uint32_t own_all[WPB][64];
  const int lane = threadIdx.x & 63;
  const int wib = wave_in_block();
  uint32_t* own = own_all[wib];
  const int W = st.W;
  const int cur = p.round & 1;
  uint64_t* __restrict__ Eo = st.E[cur];
  const uint64_t* __restrict__ AWc = st.AW[cur];
  const uint32_t k = K > 0 ? (uint32_t)K : (uint32_t)p.fanout;
  uint64_t pushed = 0;
  for (int64_t i = (int64_t)blockIdx.x * WPB + wib; i < n_wide; i += (int64_t)gridDim.x * WPB) {
    const int64_t v = ldc(wide + i);
    if (!((ldc(st.A[cur] + (v >> 5)) >> (v & 31)) & 1u)) continue;
    const int64_t rb = ldc(g.rowptr + v);
    const uint32_t deg = (uint32_t)(ldc(g.rowptr + v + 1) - rb);
    const uint64_t am = AWc ? ldc(AWc + v) : (W >= 64 ? ~0ull : (1ull << W) - 1ull);
    const uint32_t gv = gidx_s(g, v);
    // lane = word of the row
    const uint64_t f = lane < W && ((am >> lane) & 1ull) ? st.F[cur][v * W + lane] : 0ull;
    const uint32_t pos_w = AWc ? (uint32_t)__popcll(am & ((1ull << lane) - 1ull)) : (uint32_t)lane;
    const uint32_t bc = (uint32_t)__popcll(f);
    const uint32_t binc = wave_scan_u32(bc);
    const uint32_t bpos = binc - bc;
    const uint32_t btot = (uint32_t)__builtin_amdgcn_readlane((int)binc, 63);
    for (uint32_t b0 = 0; b0 < btot; b0 += 64) {
      // lane = bit b0 + lane of the row (owner lane = its word)
      const int ow = pass_owner(own, lane, bpos, bc, b0);
      const uint32_t gpos = bperm(ow, bpos), epos = bperm(ow, pos_w);
      const uint64_t gf = bperm64(ow, f);
      if (b0 + (uint32_t)lane < btot) {
        const uint32_t b = select_bit64(gf, b0 + (uint32_t)lane - gpos);
        const uint32_t mg = p.msg_base + (uint32_t)ow * 64u + b;
        uint32_t pk[K > 0 ? K : 16];
        if constexpr (K > 0)
          gossip_picks_t<K>((uint32_t)p.round, gv, mg, deg, p.gseed_lo, p.gseed_hi, pk);
        else
          gossip_picks((uint32_t)p.round, gv, mg, deg, (int)k, p.gseed_lo, p.gseed_hi, pk);
        uint64_t old[K > 0 ? K : 16];  // (K > 0: constant trip counts, unrolled)
        for (uint32_t q = 0; q < (K > 0 ? (uint32_t)K : k); ++q) {
          old[q] = 1ull;  // (not counted)
          const int64_t slot = rb + (int64_t)pk[q];
          if (CHURN && churn_dropped((uint32_t)p.round, gv, gidx(g, g.colidx[slot]), p.churn_thr,
                                     p.cseed_lo, p.cseed_hi))
            continue;  // a lost send: the connection's row stays zero
          old[q] = atomicOr((unsigned long long*)at_row(Eo, g.rev[slot], W) + epos, 1ull << b);
        }
        // the returned words are used only after all picks are issued (one wait, not k)
        for (uint32_t q = 0; q < (K > 0 ? (uint32_t)K : k); ++q) pushed += old[q] == 0ull ? 1u : 0u;
      }
    }
  }
  uint64_t c[STAT_N] = {0, 0, 0, 0, 0, 0, 0, 0};
  c[ST_SCATTER] = pushed;
  flush_stats(st.stats, c, lane);
}

}  // namespace

bool gossip_scatter_sparse_supported(const DevState& st) {
  return st.W >= 1 && st.W <= 64 && (st.AW[0] != nullptr || st.W <= PACK_W_MAX_PLAIN);
}

int64_t sparse_chunks(int64_t V) { return (((V + 31) >> 5) + SW_TASKS - 1) / SW_TASKS; }

hipError_t launch_gossip_scatter_sparse(const DevGraph& g, const DevState& st,
                                        const RoundParams& p, int64_t expect,
                                        const SparseBufs& b, hipStream_t s) {
  if (!gossip_scatter_sparse_supported(st) || b.cap < 1) return hipErrorInvalidValue;
  const int64_t chunks = sparse_chunks(g.V);
  // up to 8192 blocks (32 waves per CU over a launch; grid_max() is 2048): the push waits on its
  // atomics' round trips, and 4x the waves in flight took the sparse class 15.5 -> 14.9 ms per
  // c4 step (profiles/r05/ab_grid_max.txt, _r05u)
  auto sgrid = [](int64_t tasks) {
    return (int)std::min<int64_t>(grid_tasks_uncapped(tasks), (int64_t)SPARSE_GRID_MAX);
  };
  const int wgrid = sgrid(chunks);
  hipLaunchKernelGGL(k_sparse_words<false>, dim3(wgrid), dim3(256), 0, s, g, st, p, b);
  hipLaunchKernelGGL(k_chunk_scan, dim3(1), dim3(1024), 0, s, chunks, b);
  hipLaunchKernelGGL(k_sparse_words<true>, dim3(wgrid), dim3(256), 0, s, g, st, p, b);
  const int grid = sgrid((expect + 63) >> 6);  // 64 listed words per wave pass
  const bool ch = p.churn_thr != 0;
#define P2PG_SPARSE(CH, KK) \
  hipLaunchKernelGGL((k_sparse_push<CH, KK>), dim3(grid), dim3(256), 0, s, g, st, p, b)
  switch (p.fanout) {
    case 1: if (ch) P2PG_SPARSE(true, 1); else P2PG_SPARSE(false, 1); break;
    case 2: if (ch) P2PG_SPARSE(true, 2); else P2PG_SPARSE(false, 2); break;
    case 3: if (ch) P2PG_SPARSE(true, 3); else P2PG_SPARSE(false, 3); break;
    case 4: if (ch) P2PG_SPARSE(true, 4); else P2PG_SPARSE(false, 4); break;
    default: if (ch) P2PG_SPARSE(true, 0); else P2PG_SPARSE(false, 0); break;
  }
#undef P2PG_SPARSE
  const int64_t ntasks = (g.V + 31) >> 5;
  hipLaunchKernelGGL(k_touched_bits, dim3((unsigned)std::min<int64_t>((ntasks + 255) / 256, 4096)),
                     dim3(256), 0, s, g.V, st.T[(p.round & 1) ^ 1], b.touched);
  return hipGetLastError();
}

hipError_t launch_wide_push_e(const DevGraph& g, const DevState& st, const RoundParams& p,
                              const int64_t* items, int64_t n_items, const int32_t* wide,
                              int64_t n_wide, hipStream_t s) {
  if (st.W > 64 || (st.W > PACK_W_MAX_PLAIN && !st.AW[p.round & 1])) return hipErrorInvalidValue;
  if (n_items <= 0 || n_wide <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_wide_zero, dim3(grid_tasks((n_items + 3) >> 2)), dim3(256), 0, s, g, st,
                     p, items, n_items);
  const int grid = grid_tasks(n_wide);
  const bool ch = p.churn_thr != 0;
#define P2PG_WIDE(CH, KK) \
  hipLaunchKernelGGL((k_wide_push<CH, KK>), dim3(grid), dim3(256), 0, s, g, st, p, wide, n_wide)
  switch (p.fanout) {
    case 1: if (ch) P2PG_WIDE(true, 1); else P2PG_WIDE(false, 1); break;
    case 2: if (ch) P2PG_WIDE(true, 2); else P2PG_WIDE(false, 2); break;
    case 3: if (ch) P2PG_WIDE(true, 3); else P2PG_WIDE(false, 3); break;
    case 4: if (ch) P2PG_WIDE(true, 4); else P2PG_WIDE(false, 4); break;
    default: if (ch) P2PG_WIDE(true, 0); else P2PG_WIDE(false, 0); break;
  }
#undef P2PG_WIDE
  return hipGetLastError();
}

}  // namespace p2pg
