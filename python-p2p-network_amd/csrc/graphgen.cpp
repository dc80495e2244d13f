// Host-side peer-graph construction for the relay engine: deterministic synthetic topologies
// (counter-based Philox streams, so every rank of a multi-GPU job builds the same graph) and
// the undirected-CSR builder.
//
// What it stands in for: in p2pnetwork the topology is whatever Node.connect_with_node calls an
// application makes (p2pnetwork/node.py:122-176); every TCP connection is usable in both
// directions for relay because Node.all_nodes = nodes_inbound + nodes_outbound
// (node.py:75-78), self-connections are refused (node.py:131-133, :153) and duplicate
// connections are refused (node.py:136-139, :153).  Hence: undirected simple graph, CSR with
// ascending neighbour ids (the lowest-id tie-break order), no self loops, no multi-edges.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/p2pgpu.h"
#include "internal.h"
#include "philox.h"

struct p2pg_graph {
  int64_t V = 0;
  std::vector<int64_t> rowptr;
  std::vector<int32_t> colidx;
};

namespace p2pg {

thread_local std::string g_error;
void set_global_error(const std::string& s) { g_error = s; }

namespace {

// Sequential Philox stream: block i = philox(ctr=(i_lo, i_hi, stream, tag), key).
struct Stream {
  uint32_t k0, k1, stream, tag;
  uint64_t block = 0;
  u32x4 buf{};
  int used = 4;
  Stream(uint64_t seed, uint32_t tag_, uint32_t stream_)
      : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), stream(stream_), tag(tag_) {}
  uint32_t next() {
    if (used == 4) {
      u32x4 c = {(uint32_t)block, (uint32_t)(block >> 32), stream, tag};
      buf = philox4x32_10(c, k0, k1);
      ++block;
      used = 0;
    }
    return word_of(buf, used++);
  }
  // uniform double in (0, 1)
  double uniform() { return ((double)next() + 0.5) * (1.0 / 4294967296.0); }
};

bool build_csr(int64_t V, const std::vector<int32_t>& a, const std::vector<int32_t>& b,
               p2pg_graph* g) {
  const int64_t n = (int64_t)a.size();
  std::vector<int64_t> deg(V + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (a[i] == b[i]) continue;
    deg[a[i]]++;
    deg[b[i]]++;
  }
  std::vector<int64_t> start(V + 1, 0);
  for (int64_t v = 0; v < V; ++v) start[v + 1] = start[v] + deg[v];
  std::vector<int32_t> col(start[V]);
  std::vector<int64_t> cur(start.begin(), start.end() - 1);
  for (int64_t i = 0; i < n; ++i) {
    if (a[i] == b[i]) continue;
    col[cur[a[i]]++] = b[i];
    col[cur[b[i]]++] = a[i];
  }
  // sort + dedup each row in parallel, then compact
  std::vector<int64_t> keep(V, 0);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t v = 0; v < V; ++v) {
    int32_t* s = col.data() + start[v];
    int32_t* e = col.data() + start[v + 1];
    std::sort(s, e);
    keep[v] = std::unique(s, e) - s;
  }
  g->V = V;
  g->rowptr.assign(V + 1, 0);
  for (int64_t v = 0; v < V; ++v) g->rowptr[v + 1] = g->rowptr[v] + keep[v];
  g->colidx.resize(g->rowptr[V]);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t v = 0; v < V; ++v)
    std::memcpy(g->colidx.data() + g->rowptr[v], col.data() + start[v], keep[v] * sizeof(int32_t));
  return true;
}

inline uint64_t ekey(uint32_t x, uint32_t y) {
  return x < y ? ((uint64_t)x << 32 | y) : ((uint64_t)y << 32 | x);
}

// Random d-regular graph: stub pairing in rounds; unsuitable pairs (self loop / existing
// edge) go back into the pool, which is reshuffled; a round without progress restarts the
// attempt with the next Philox stream.
bool gen_random_regular(int64_t V, int d, uint64_t seed, std::vector<int32_t>& A,
                        std::vector<int32_t>& B) {
  if (d < 0 || d >= V || ((V * d) & 1)) {
    set_global_error("random_regular: need 0 <= d < V and V*d even");
    return false;
  }
  for (uint32_t attempt = 0; attempt < 1000; ++attempt) {
    Stream rs(seed, TAG_RRG, attempt);
    std::vector<int32_t> stubs;
    stubs.reserve(V * d);
    for (int64_t v = 0; v < V; ++v)
      for (int i = 0; i < d; ++i) stubs.push_back((int32_t)v);
    std::unordered_set<uint64_t> edges;
    edges.reserve(V * d);
    A.clear();
    B.clear();
    std::vector<int32_t> left;
    while (!stubs.empty()) {
      for (int64_t i = (int64_t)stubs.size() - 1; i > 0; --i) {
        int64_t j = lemire32(rs.next(), (uint32_t)(i + 1));
        std::swap(stubs[i], stubs[j]);
      }
      left.clear();
      bool progress = false;
      for (size_t i = 0; i + 1 < stubs.size(); i += 2) {
        int32_t x = stubs[i], y = stubs[i + 1];
        if (x != y && edges.insert(ekey(x, y)).second) {
          A.push_back(x);
          B.push_back(y);
          progress = true;
        } else {
          left.push_back(x);
          left.push_back(y);
        }
      }
      if (!progress) break;
      stubs.swap(left);
    }
    if (stubs.empty()) return true;
  }
  set_global_error("random_regular: no simple graph after 1000 attempts");
  return false;
}

// G(n,p) by geometric skipping over the lower triangle (Batagelj & Brandes 2005).
bool gen_gnp(int64_t V, double mean_deg, uint64_t seed, std::vector<int32_t>& A,
             std::vector<int32_t>& B) {
  if (V < 2) return true;
  const double p = mean_deg / (double)(V - 1);
  if (!(p > 0.0) || p >= 1.0) {
    set_global_error("gnp: need 0 < mean_degree < V-1");
    return false;
  }
  Stream rs(seed, TAG_GNP, 0);
  const double lp = std::log1p(-p);
  int64_t v = 1, w = -1;
  A.reserve((size_t)(mean_deg * V / 2 * 1.01) + 16);
  B.reserve(A.capacity());
  while (v < V) {
    const double r = rs.uniform();
    w += 1 + (int64_t)std::floor(std::log1p(-r) / lp);
    while (w >= v && v < V) {
      w -= v;
      ++v;
    }
    if (v < V) {
      A.push_back((int32_t)v);
      B.push_back((int32_t)w);
    }
  }
  return true;
}

// Barabasi-Albert preferential attachment, linear time (endpoint list sampling), initial
// (m+1)-clique; each new vertex attaches to m distinct existing vertices.
bool gen_ba(int64_t V, int m, uint64_t seed, std::vector<int32_t>& A, std::vector<int32_t>& B) {
  if (m < 1 || V <= m) {
    set_global_error("barabasi_albert: need 1 <= m < V");
    return false;
  }
  std::vector<int32_t> ends;
  ends.reserve((size_t)2 * m * V);
  A.reserve((size_t)m * V);
  B.reserve((size_t)m * V);
  for (int x = 0; x <= m; ++x)
    for (int y = x + 1; y <= m; ++y) {
      A.push_back(x);
      B.push_back(y);
      ends.push_back(x);
      ends.push_back(y);
    }
  Stream rs(seed, TAG_BAG, 0);
  std::vector<int32_t> pick(m);
  for (int64_t v = m + 1; v < V; ++v) {
    int got = 0;
    const uint32_t n = (uint32_t)ends.size();
    while (got < m) {
      int32_t t = ends[lemire32(rs.next(), n)];
      bool dup = false;
      for (int q = 0; q < got; ++q) dup |= (pick[q] == t);
      if (!dup) pick[got++] = t;
    }
    for (int q = 0; q < m; ++q) {
      A.push_back((int32_t)v);
      B.push_back(pick[q]);
      ends.push_back((int32_t)v);
      ends.push_back(pick[q]);
    }
  }
  return true;
}

// Watts-Strogatz small world: ring lattice v ~ v+1..v+k/2; each lattice edge is rewired with
// probability beta to a uniform target outside v's lattice window (pure function of
// (v, j, attempt) -> parallel and rank-independent); rewired duplicates merge in the CSR.
bool gen_ws(int64_t V, int k, double beta, uint64_t seed, std::vector<int32_t>& A,
            std::vector<int32_t>& B) {
  if (k < 2 || (k & 1) || k >= V || beta < 0.0 || beta > 1.0) {
    set_global_error("watts_strogatz: need even 2 <= k < V and 0 <= beta <= 1");
    return false;
  }
  const int h = k / 2;
  const uint32_t thr = beta >= 1.0 ? 0xFFFFFFFFu : (uint32_t)std::floor(beta * 4294967296.0);
  A.resize((size_t)V * h);
  B.resize((size_t)V * h);
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ TAG_WSG;
#pragma omp parallel for schedule(static)
  for (int64_t v = 0; v < V; ++v) {
    for (int j = 1; j <= h; ++j) {
      int64_t t = (v + j) % V;
      for (uint32_t att = 0; att < 16; ++att) {
        u32x4 c = {(uint32_t)v, (uint32_t)j, att, TAG_WSG};
        u32x4 r = philox4x32_10(c, k0, k1);
        if (att == 0 && !(r.x < thr || thr == 0xFFFFFFFFu)) break;  // keep lattice edge
        int64_t w = lemire32(r.y, (uint32_t)V);
        int64_t dist = w > v ? w - v : v - w;
        dist = std::min(dist, V - dist);
        if (dist > h) {
          t = w;
          break;
        }
      }
      A[(size_t)v * h + (j - 1)] = (int32_t)v;
      B[(size_t)v * h + (j - 1)] = (int32_t)t;
    }
  }
  return true;
}

// Config 1: ring 0-1-..-(V-1)-0 plus chords (i, i+stride) for i = 0, stride, 2*stride, ...
bool gen_ring_chords(int64_t V, int stride, std::vector<int32_t>& A, std::vector<int32_t>& B) {
  if (V < 3) {
    set_global_error("ring_chords: need V >= 3");
    return false;
  }
  for (int64_t v = 0; v < V; ++v) {
    A.push_back((int32_t)v);
    B.push_back((int32_t)((v + 1) % V));
  }
  if (stride > 1)
    for (int64_t v = 0; v + stride < V; v += stride) {
      A.push_back((int32_t)v);
      B.push_back((int32_t)(v + stride));
    }
  return true;
}

}  // namespace
}  // namespace p2pg

using namespace p2pg;

extern "C" {

int p2pg_graph_generate(int32_t kind, int64_t V, double a, double b, uint64_t seed,
                        p2pg_graph** out) {
  if (!out || V <= 0 || V > 0x7FFFFFFFll) {
    set_global_error("graph_generate: bad arguments");
    return P2PG_ERR_ARG;
  }
  *out = nullptr;
  std::vector<int32_t> A, B;
  bool ok = false;
  try {
    switch (kind) {
      case 0: ok = gen_random_regular(V, (int)a, seed, A, B); break;
      case 1: ok = gen_gnp(V, a, seed, A, B); break;
      case 2: ok = gen_ba(V, (int)a, seed, A, B); break;
      case 3: ok = gen_ws(V, (int)a, b, seed, A, B); break;
      case 4: ok = gen_ring_chords(V, (int)a, A, B); break;
      default: set_global_error("graph_generate: unknown kind"); return P2PG_ERR_ARG;
    }
    if (!ok) return P2PG_ERR_GRAPH;
    p2pg_graph* g = new p2pg_graph;
    build_csr(V, A, B, g);
    *out = g;
  } catch (const std::bad_alloc&) {
    set_global_error("graph_generate: out of host memory");
    return P2PG_ERR_NOMEM;
  }
  return P2PG_OK;
}

int p2pg_graph_from_edges(int64_t V, int64_t n_edges, const int32_t* src, const int32_t* dst,
                          p2pg_graph** out) {
  if (!out || V <= 0 || V > 0x7FFFFFFFll || n_edges < 0 || (n_edges > 0 && (!src || !dst))) {
    set_global_error("graph_from_edges: bad arguments");
    return P2PG_ERR_ARG;
  }
  *out = nullptr;
  for (int64_t i = 0; i < n_edges; ++i)
    if (src[i] < 0 || src[i] >= V || dst[i] < 0 || dst[i] >= V) {
      set_global_error("graph_from_edges: endpoint out of range");
      return P2PG_ERR_GRAPH;
    }
  try {
    std::vector<int32_t> A(src, src + n_edges), B(dst, dst + n_edges);
    p2pg_graph* g = new p2pg_graph;
    build_csr(V, A, B, g);
    *out = g;
  } catch (const std::bad_alloc&) {
    set_global_error("graph_from_edges: out of host memory");
    return P2PG_ERR_NOMEM;
  }
  return P2PG_OK;
}

int p2pg_graph_info(const p2pg_graph* g, int64_t* V, int64_t* nnz) {
  if (!g) return P2PG_ERR_ARG;
  if (V) *V = g->V;
  if (nnz) *nnz = (int64_t)g->colidx.size();
  return P2PG_OK;
}

int p2pg_graph_arrays(const p2pg_graph* g, const int64_t** rowptr, const int32_t** colidx) {
  if (!g) return P2PG_ERR_ARG;
  if (rowptr) *rowptr = g->rowptr.data();
  if (colidx) *colidx = g->colidx.data();
  return P2PG_OK;
}

void p2pg_graph_free(p2pg_graph* g) { delete g; }

int p2pg_make_sources(int64_t V, int32_t M, uint64_t seed, uint32_t msg_id_base, int32_t* src) {
  if (V <= 0 || V > 0x7FFFFFFFll || M < 0 || (M > 0 && !src)) {
    set_global_error("make_sources: bad arguments");
    return P2PG_ERR_ARG;
  }
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32) ^ TAG_SRC;
  for (int32_t m = 0; m < M; ++m) {
    u32x4 c = {msg_id_base + (uint32_t)m, 0, 0, 0};
    src[m] = (int32_t)lemire32(philox4x32_10(c, k0, k1).x, (uint32_t)V);
  }
  return P2PG_OK;
}

void p2pg_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  u32x4 c = {ctr[0], ctr[1], ctr[2], ctr[3]};
  u32x4 r = philox4x32_10(c, key[0], key[1]);
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
  out[3] = r.w;
}

int p2pg_gossip_targets(uint32_t round, uint32_t peer, uint32_t msg, uint32_t deg, int32_t k,
                        uint64_t seed, uint32_t* out) {
  if (k < 1 || k > 16 || (deg > 0 && !out)) {
    set_global_error("gossip_targets: need 1 <= k <= 16 and an output array");
    return P2PG_ERR_ARG;
  }
  if (deg <= (uint32_t)k) {  // every connection, in adjacency order
    for (uint32_t j = 0; j < deg; ++j) out[j] = j;
    return (int)deg;
  }
  const uint32_t s0 = (uint32_t)seed, s1 = (uint32_t)(seed >> 32);
  // k <= 4: the folded-round Philox of the device's dense pushes (philox_pick), else the generic
  if (k <= 4) {
    const PickKey key = pick_key(round, peer, s0, s1);
    uint32_t t[4];
    switch (k) {
      case 1: { uint32_t o[1]; gossip_picks_k<1>(key, msg, deg, o); t[0] = o[0]; break; }
      case 2: { uint32_t o[2]; gossip_picks_k<2>(key, msg, deg, o); t[0] = o[0]; t[1] = o[1]; break; }
      case 3: { uint32_t o[3]; gossip_picks_k<3>(key, msg, deg, o); for (int i = 0; i < 3; ++i) t[i] = o[i]; break; }
      default: { uint32_t o[4]; gossip_picks_k<4>(key, msg, deg, o); for (int i = 0; i < 4; ++i) t[i] = o[i]; break; }
    }
    for (int i = 0; i < k; ++i) out[i] = t[i];
    return k;
  }
  gossip_picks(round, peer, msg, deg, k, s0, s1, out);
  return k;
}

int p2pg_churn_lost(uint32_t round, uint32_t a, uint32_t b, uint32_t threshold, uint64_t seed) {
  return churn_dropped(round, a, b, threshold, (uint32_t)seed, (uint32_t)(seed >> 32)) ? 1 : 0;
}

const char* p2pg_global_error(void) { return g_error.c_str(); }

}  // extern "C"
