/*
 * relay_oracle.c -- plain-C restatement of the p2pnetwork flood relay (ORACLE: test
 * infrastructure only; built into oracle/_build/liboracle.so by oracle/Makefile).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker or as the timed CPU baseline ("kind": "port").
 *
 * Restates (pj8912/python-p2p-network):
 *   Node.send_to_nodes(data, exclude=[sender])  p2pnetwork/node.py:106-112: a relay to every
 *     connection but the sender; Node.send_to_node counts message_count_send first
 *     (node.py:114-120, :116); neighbours = Node.all_nodes (node.py:75-78); the app-level dedup
 *     of README.md:20 (forward first receipts only).  Round-synchronous with lowest-id sender
 *     as parent; push-gossip and churn as defined in SURVEY.md A.3 / A.4.
 * Independent of the engine's code: its own Philox, a per-peer-word pull for flood (every
 * frontier row rewritten each round, no activity bitmaps), atomic-OR pushes for gossip.
 * Pinned by tests/test_oracle_golden.py against the reference-harness fixtures.
 *
 * seen_out (optional, [V][W] uint64): every peer's seen set at quiescence.
 * stats[r*8 + i]: 0 new deliveries, 1 relays, 2 active peers, 3 active words, 4 wedges,
 * 5 deg of active peers, 6 gossip scatter words, 7 unused.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint32_t x, y, z, w; } q4;

static q4 ph10(q4 c, uint32_t k0, uint32_t k1) {
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    q4 n = {(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1,
            (uint32_t)p0};
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

static int dropped(uint32_t r, uint32_t a, uint32_t b, uint32_t thr, uint64_t seed) {
  if (!thr) return 0;
  q4 c = {r, a < b ? a : b, a < b ? b : a, 0x0043484Eu};
  return ph10(c, (uint32_t)seed, (uint32_t)(seed >> 32)).x < thr;
}

/* k distinct indices of [0, n) (n > k): Floyd with Lemire, word i%4 of block i/4 */
static void picks(uint32_t r, uint32_t v, uint32_t m, uint32_t n, int k, uint64_t seed,
                  uint32_t* out) {
  q4 b = {0, 0, 0, 0};
  for (int i = 0; i < k; ++i) {
    if ((i & 3) == 0) {
      q4 c = {r, v, m, 0x00475350u | ((uint32_t)(i >> 2) << 24)};
      b = ph10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    }
    uint32_t word = (i & 3) == 0 ? b.x : (i & 3) == 1 ? b.y : (i & 3) == 2 ? b.z : b.w;
    uint32_t jmax = n - (uint32_t)k + (uint32_t)i;
    uint32_t t = (uint32_t)(((uint64_t)word * (uint64_t)(jmax + 1u)) >> 32);
    int dup = 0;
    for (int q = 0; q < i; ++q) dup |= out[q] == t;
    out[i] = dup ? jmax : t;
  }
}

static uint64_t fullmask(int64_t w, int64_t W, int32_t M) {
  return (w < W - 1 || (M & 63) == 0) ? ~0ull : ((1ull << (M & 63)) - 1ull);
}

static void round0(int64_t V, const int64_t* rp, int32_t M, const int32_t* src, int64_t W,
                   uint64_t* seen, uint64_t* F, int gossip, int k, uint64_t* st,
                   int32_t* hop, int32_t* par) {
  memset(F, 0, sizeof(uint64_t) * V * W);
  for (int32_t m = 0; m < M; ++m) {
    int64_t v = src[m];
    F[v * W + (m >> 6)] |= 1ull << (m & 63);
    seen[v * W + (m >> 6)] |= 1ull << (m & 63);
    int64_t d = rp[v + 1] - rp[v];
    st[0] += 1;
    st[1] += gossip ? (uint64_t)(d < k ? d : k) : (uint64_t)d;
    if (hop) {
      hop[v * M + m] = 0;
      par[v * M + m] = -1;
    }
  }
  for (int64_t v = 0; v < V; ++v) {
    int any = 0;
    for (int64_t w = 0; w < W; ++w)
      if (F[v * W + w]) {
        any = 1;
        st[3] += 1;
        st[4] += (uint64_t)(rp[v + 1] - rp[v]);
      }
    if (any) {
      st[2] += 1;
      st[5] += (uint64_t)(rp[v + 1] - rp[v]);
    }
  }
}

int oracle_flood(int64_t V, const int64_t* rp, const int32_t* ci, int32_t M, const int32_t* src,
                 uint32_t churn_thr, uint64_t churn_seed, int32_t max_rounds, uint64_t* stats,
                 int32_t* n_rounds, int32_t* hop, int32_t* par, uint64_t* seen_out) {
  const int64_t W = (M + 63) / 64;
  uint64_t* seen = calloc((size_t)(V * W), 8);
  uint64_t* F = calloc((size_t)(V * W), 8);
  uint64_t* Fn = calloc((size_t)(V * W), 8);
  if (!seen || !F || !Fn) {
    free(seen), free(F), free(Fn);
    return -4;
  }
  if (hop) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < V * M; ++i) hop[i] = par[i] = -1;
  }
  memset(stats, 0, sizeof(uint64_t) * 8 * (size_t)max_rounds);
  round0(V, rp, M, src, W, seen, F, 0, 0, stats, hop, par);
  int32_t r = 1;
  for (; r < max_rounds; ++r) {
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0;
#pragma omp parallel
    {
      uint64_t* acc = malloc(sizeof(uint64_t) * W);
#pragma omp for schedule(dynamic, 256) reduction(+ : s0, s1, s2, s3, s4, s5)
      for (int64_t u = 0; u < V; ++u) {
        const int64_t d = rp[u + 1] - rp[u];
        memset(acc, 0, sizeof(uint64_t) * W);
        for (int64_t e = rp[u]; e < rp[u + 1]; ++e) {
          const int64_t v = ci[e];
          uint64_t any_v = 0; /* nothing sent by v: no churn draw needed */
          for (int64_t w = 0; w < W; ++w) any_v |= F[v * W + w];
          if (!any_v) continue;
          if (dropped((uint32_t)(r - 1), (uint32_t)u, (uint32_t)v, churn_thr, churn_seed)) continue;
          for (int64_t w = 0; w < W; ++w) acc[w] |= F[v * W + w];
        }
        int any = 0;
        for (int64_t w = 0; w < W; ++w) {
          const uint64_t nw = acc[w] & ~seen[u * W + w] & fullmask(w, W, M);
          Fn[u * W + w] = nw;
          if (!nw) continue;
          seen[u * W + w] |= nw;
          any = 1;
          const uint64_t pc = (uint64_t)__builtin_popcountll(nw);
          s0 += pc;
          s1 += pc * (uint64_t)(d - 1);
          s3 += 1;
          s4 += (uint64_t)d;
          if (hop) {
            uint64_t pend = nw;
            for (int64_t e = rp[u]; e < rp[u + 1] && pend; ++e) {
              const int64_t v = ci[e];
              if (!(F[v * W + w] & pend)) continue;
              if (dropped((uint32_t)(r - 1), (uint32_t)u, (uint32_t)v, churn_thr, churn_seed)) continue;
              uint64_t hit = F[v * W + w] & pend;
              pend &= ~hit;
              while (hit) {
                const int b = __builtin_ctzll(hit);
                hit &= hit - 1;
                hop[u * M + w * 64 + b] = r;
                par[u * M + w * 64 + b] = (int32_t)v;
              }
            }
          }
        }
        if (any) {
          s2 += 1;
          s5 += (uint64_t)d;
        }
      }
      free(acc);
    }
    uint64_t* st = stats + 8 * (size_t)r;
    st[0] = s0, st[1] = s1, st[2] = s2, st[3] = s3, st[4] = s4, st[5] = s5;
    uint64_t* t = F;
    F = Fn;
    Fn = t;
    if (!s0) {
      ++r;
      break;
    }
  }
  *n_rounds = r;
  if (seen_out) memcpy(seen_out, seen, sizeof(uint64_t) * (size_t)(V * W));
  free(seen), free(F), free(Fn);
  return 0;
}

static int cmp_u64(const void* a, const void* b) {
  uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}

int oracle_gossip(int64_t V, const int64_t* rp, const int32_t* ci, int32_t M,
                  const int32_t* src, int32_t k, uint64_t gseed, uint32_t msg_base,
                  uint32_t churn_thr, uint64_t churn_seed, int32_t max_rounds, uint64_t* stats,
                  int32_t* n_rounds, int32_t* hop, int32_t* par, uint64_t* seen_out) {
  const int64_t W = (M + 63) / 64;
  uint64_t* seen = calloc((size_t)(V * W), 8);
  uint64_t* F = calloc((size_t)(V * W), 8);
  uint64_t* nx = calloc((size_t)(V * W), 8);
  int32_t* cand = hop ? malloc(sizeof(int32_t) * (size_t)(V * M)) : NULL;
  if (!seen || !F || !nx || (hop && !cand)) {
    free(seen), free(F), free(nx), free(cand);
    return -4;
  }
  if (hop) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < V * M; ++i) hop[i] = par[i] = -1, cand[i] = 0x7FFFFFFF;
  }
  memset(stats, 0, sizeof(uint64_t) * 8 * (size_t)max_rounds);
  round0(V, rp, M, src, W, seen, F, 1, k, stats, hop, par);
  int32_t r = 0;
  for (;;) {
    /* pushes made in round r by its first receipts */
    uint64_t scat = 0, active = 0;
#pragma omp parallel
    {
      uint64_t* tg = malloc(sizeof(uint64_t) * 64 * 16);
      uint32_t pk[16];
#pragma omp for schedule(dynamic, 256) reduction(+ : scat, active)
      for (int64_t v = 0; v < V; ++v) {
        const int64_t d = rp[v + 1] - rp[v];
        for (int64_t w = 0; w < W; ++w) {
          uint64_t f = F[v * W + w];
          if (!f) continue;
          active += 1;
          int nt = 0;
          while (f) {
            const int b = __builtin_ctzll(f);
            f &= f - 1;
            const uint32_t m = (uint32_t)(w * 64 + b);
            int cnt = d <= k ? (int)d : k;
            if (d > k) picks((uint32_t)r, (uint32_t)v, msg_base + m, (uint32_t)d, k, gseed, pk);
            for (int q = 0; q < cnt; ++q) {
              const int64_t t = ci[rp[v] + (d <= k ? q : (int64_t)pk[q])];
              if (dropped((uint32_t)r, (uint32_t)v, (uint32_t)t, churn_thr, churn_seed)) continue;
              __atomic_fetch_or(&nx[t * W + w], 1ull << b, __ATOMIC_RELAXED);
              if (cand) {
                int32_t* c = &cand[t * M + m];
                int32_t old = __atomic_load_n(c, __ATOMIC_RELAXED);
                while ((int32_t)v < old &&
                       !__atomic_compare_exchange_n(c, &old, (int32_t)v, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
                }
              }
              tg[nt++] = (uint64_t)t;
            }
          }
          qsort(tg, (size_t)nt, sizeof(uint64_t), cmp_u64);
          for (int i = 0; i < nt; ++i) scat += (i == 0 || tg[i] != tg[i - 1]);
        }
      }
      free(tg);
    }
    stats[8 * (size_t)r + 6] = scat;
    if (!active || r + 1 >= max_rounds) {
      ++r;
      break;
    }
    ++r;
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : s0, s1, s2, s3, s4, s5)
    for (int64_t u = 0; u < V; ++u) {
      const int64_t d = rp[u + 1] - rp[u];
      const uint64_t fan = (uint64_t)(d < k ? d : k);
      int any = 0;
      for (int64_t w = 0; w < W; ++w) {
        const uint64_t x = nx[u * W + w];
        nx[u * W + w] = 0;
        const uint64_t nw = x & ~seen[u * W + w];
        if (cand) { /* candidates of pushed-but-seen bits are stale: re-arm them */
          uint64_t h = x & ~nw;
          while (h) {
            const int b = __builtin_ctzll(h);
            h &= h - 1;
            cand[u * M + w * 64 + b] = 0x7FFFFFFF;
          }
        }
        F[u * W + w] = nw;
        if (!nw) continue;
        seen[u * W + w] |= nw;
        any = 1;
        const uint64_t pc = (uint64_t)__builtin_popcountll(nw);
        s0 += pc, s1 += pc * fan, s3 += 1, s4 += (uint64_t)d;
        if (hop) {
          uint64_t h = nw;
          while (h) {
            const int b = __builtin_ctzll(h);
            h &= h - 1;
            hop[u * M + w * 64 + b] = r;
            par[u * M + w * 64 + b] = cand[u * M + w * 64 + b];
            cand[u * M + w * 64 + b] = 0x7FFFFFFF;
          }
        }
      }
      if (any) s2 += 1, s5 += (uint64_t)d;
    }
    uint64_t* st = stats + 8 * (size_t)r;
    st[0] = s0, st[1] = s1, st[2] = s2, st[3] = s3, st[4] = s4, st[5] = s5;
  }
  *n_rounds = r;
  if (seen_out) memcpy(seen_out, seen, sizeof(uint64_t) * (size_t)(V * W));
  free(seen), free(F), free(nx), free(cand);
  return 0;
}
