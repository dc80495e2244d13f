/*
 * p2pgpu.h -- C-ABI of the MI355X broadcast/relay engine (libp2pgpu.so).
 *
 * The engine replaces, for ONE hot path, what a p2pnetwork application does with
 * Node.send_to_nodes + node_message + a message-id "seen" set (the dedup/no-echo contract of
 * /root/reference/README.md:20): it runs that flood relay, and a push-gossip variant, over a
 * whole simulated peer graph at once, 64 concurrent broadcasts per uint64 bitset word.
 *
 * Reference interface each entry point replaces (file:line in pj8912/python-p2p-network):
 *   p2pg_load_csr / p2pg_graph_*  <- the topology built by Node.connect_with_node
 *                                    (p2pnetwork/node.py:122-176); a peer's neighbour list is
 *                                    Node.all_nodes = nodes_inbound + nodes_outbound (node.py:75-78)
 *   p2pg_set_sources              <- the originating Node.send_to_nodes(data) call per broadcast
 *                                    (node.py:106-112)
 *   p2pg_step / p2pg_run          <- one / all rounds of: NodeConnection.run receive loop
 *                                    (nodeconnection.py:186-218) -> Node.node_message
 *                                    (node.py:334-338) -> app dedup -> send_to_nodes(data,
 *                                    exclude=[sender]) (node.py:106-112) -> send_to_node
 *                                    (node.py:114-120, message_count_send += 1 at :116)
 *   p2pg_round_stats.relays       <- sum over peers of Node.message_count_send (node.py:65,116)
 *   p2pg_get_new_deliveries       <- the node_message(node, data) events of one round, as
 *                                    (peer, msg, hop, parent) records (node.py:334-338)
 *   p2pg_get_sends                <- every Node.send_to_node call of one round (node.py:114-120),
 *                                    i.e. every packet NodeConnection.run hands to node_message
 *                                    the next round (nodeconnection.py:211-216), duplicates
 *                                    included, with the ones churn loses (nodeconnection.py:123-126)
 *   p2pg_drop_relays              <- an app whose node_message did not call send_to_nodes for a
 *                                    first receipt (README.md:20: the app decides)
 *   p2pg_round_stats.received     <- sum over peers of message_count_recv (nodeconnection.py:215)
 *   p2pg_read_planes              <- each app's "seen" set + first-receipt (hop, sender)
 *   p2pg_last_error               <- (reference swallows errors via debug_print, node.py:80-83)
 *
 * Conventions: plain C types only; 0 = OK, negative = error (message via p2pg_last_error);
 * no exceptions cross the ABI; the engine owns all device memory; caller keeps ownership of
 * every host array it passes; one engine per host thread (not re-entrant).
 */
#ifndef P2PGPU_H
#define P2PGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define P2PG_OK 0
#define P2PG_ERR_ARG (-1)
#define P2PG_ERR_STATE (-2)
#define P2PG_ERR_HIP (-3)
#define P2PG_ERR_NOMEM (-4)
#define P2PG_ERR_GRAPH (-5)

#define P2PG_MODE_FLOOD 0  /* forward to all connections except the sender (node.py:106-112) */
#define P2PG_MODE_GOSSIP 1 /* push-gossip: k Philox-chosen connections      */

#define P2PG_PUSH_NONE 0   /* flood, or nothing pushed                                   */
#define P2PG_PUSH_ATOMIC 1 /* gossip sparse round: row atomicOr into the targets' rows    */
#define P2PG_PUSH_EDGE 2   /* gossip dense round: per-connection mask stores (E plane)    */
#define P2PG_PUSH_FUSED 3  /* as EDGE, in one pass with this round's pull of E            */
#define P2PG_PUSH_UPDATE_EDGE 4 /* as EDGE, in one pass with this round's update (the    */
                                /* row pushes of a sparse round before it)                */

#define P2PG_FLAG_RECORD 1u /* keep hop/parent planes [V][M] (validation scale)            */
#define P2PG_FLAG_TIMING 2u /* per-kernel HIP-event timing (p2pg_kernel_times)              */
#define P2PG_FLAG_NO_AUTOSTOP 4u /* partitioned runs: keep stepping after a locally quiet
                                    round (the caller decides global quiescence)          */
#define P2PG_FLAG_LOCAL_GRAPH 8u /* rank-local graph of a vertex partition: ghost peers have
                                    empty rows, so symmetry is checked between non-empty
                                    rows only; a ghost's reverse slot is marked, so at
                                    16 < W <= 64 gossip takes the dense rounds (per-
                                    connection pushes for local connections, row pushes for
                                    ghost ones, exchanged); narrower rows: row atomics only */

#define P2PG_FLAG_RECEIVED 16u /* churn runs: count every round's lost sends, so that
                                    p2pg_round_stats.received is exact (a counting pass over the
                                    round's frontier after each round: config 5 +100 %); without
                                    it a churn run reports the sends of the round before there
                                    (an upper bound, received_exact = 0)                     */

typedef struct p2pg_engine p2pg_engine;
typedef struct p2pg_graph p2pg_graph;

typedef struct p2pg_config {
  int32_t mode;              /* P2PG_MODE_*                                              */
  int32_t fanout;            /* gossip k (1..16); ignored for flood                       */
  uint64_t gossip_seed;      /* Philox key for gossip picks                               */
  uint64_t churn_seed;       /* Philox key for the per-round edge-drop mask               */
  uint32_t churn_threshold;  /* send lost iff philox(...).x < threshold; 0 = no churn    */
  uint32_t msg_id_base;      /* global id of local message 0 (message-axis sharding)      */
  uint32_t flags;            /* P2PG_FLAG_*                                               */
  int32_t device;            /* HIP device ordinal                                        */
} p2pg_config;

typedef struct p2pg_round_stats {
  int32_t round;             /* round index r (0 = origination)                           */
  int32_t active;            /* 1 if messages are still in flight after this round        */
  uint64_t new_deliveries;   /* (peer,msg) first receipts in round r (= node_message events
                                that pass dedup)                                          */
  uint64_t relays;           /* send_to_node calls made in round r (message_count_send)   */
  uint64_t active_vertices;  /* |A_r|: peers with >= 1 first receipt in round r           */
  uint64_t active_words;     /* N_aw: nonzero (peer, word) of the round-r frontier        */
  uint64_t wedges;           /* sum over nonzero frontier words of deg(peer)              */
  uint64_t deg_active;       /* sum over A_r of deg(peer)                                 */
  uint64_t scatter_words;    /* gossip: nonzero (sender, target, word) masks pushed       */
  uint64_t touched_words;    /* gossip: nonzero pushed-to words consumed in round r       */
  int32_t push_form;         /* gossip: how round r's pushes left (P2PG_PUSH_*); flood 0    */
  int32_t received_exact;    /* 1: `received` is exact; 0: a churn run without
                                P2PG_FLAG_RECEIVED, `received` = the sends of round r-1     */
  uint64_t received;         /* packets that arrived in round r: the sends of round r-1 less
                                those lost to churn or to a connection removed in between
                                (sum over peers of message_count_recv += 1,
                                nodeconnection.py:215; duplicates included, 0 at round 0)  */
} p2pg_round_stats;

/* ---- graphs (host side; no GPU needed) ---------------------------------------------- */
/* kind: 0 random d-regular (a = d), 1 G(n,p) with p = a / (V-1) (a = mean degree),
 *       2 Barabasi-Albert (a = m, initial (m+1)-clique), 3 Watts-Strogatz (a = k, b = beta),
 *       4 ring + chords (config 1: a = chord stride, 0 = none)                           */
int p2pg_graph_generate(int32_t kind, int64_t V, double a, double b, uint64_t seed,
                        p2pg_graph** out);
/* Build from an undirected edge list (any order, duplicates/self-loops dropped). */
int p2pg_graph_from_edges(int64_t V, int64_t n_edges, const int32_t* src, const int32_t* dst,
                          p2pg_graph** out);
int p2pg_graph_info(const p2pg_graph* g, int64_t* V, int64_t* nnz);
/* Borrowed pointers, valid until p2pg_graph_free. */
int p2pg_graph_arrays(const p2pg_graph* g, const int64_t** rowptr, const int32_t** colidx);
void p2pg_graph_free(p2pg_graph* g);
/* src[m] = lemire32(philox(key=(seed_lo, seed_hi ^ 'SRC'), ctr=(msg_id_base+m,0,0,0)).x, V) */
int p2pg_make_sources(int64_t V, int32_t M, uint64_t seed, uint32_t msg_id_base, int32_t* src);
/* Host Philox4x32-10 (KAT hook). */
void p2pg_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* Host evaluation of the engine's random draws (the wire bridge replays the sends of a run):
 * the connections (indices into the peer's ascending adjacency) a gossip first receipt of
 * message msg (global id) at peer in round `round` is pushed to, in draw order -- what
 * Node.send_to_node is called on (node.py:114-120); returns their number min(k, deg).     */
int p2pg_gossip_targets(uint32_t round, uint32_t peer, uint32_t msg, uint32_t deg, int32_t k,
                        uint64_t seed, uint32_t* out);
/* 1 iff a send over {a, b} made in round `round` is lost to churn.       */
int p2pg_churn_lost(uint32_t round, uint32_t a, uint32_t b, uint32_t threshold, uint64_t seed);

/* ---- engine ------------------------------------------------------------------------- */
int p2pg_create(const p2pg_config* cfg, p2pg_engine** out);
int p2pg_load_csr(p2pg_engine* e, int64_t V, const int64_t* rowptr, const int32_t* colidx);
int p2pg_set_sources(p2pg_engine* e, int32_t M, const int32_t* src);
/* Back to round 0 with the same graph and sources (clears seen/frontier state). */
int p2pg_reset(p2pg_engine* e);
/* One round. Returns 1 while messages are in flight, 0 when quiescent, < 0 on error. */
int p2pg_step(p2pg_engine* e, p2pg_round_stats* out);
/* Rounds until quiescence or max_rounds; per_round may be NULL (else >= max_rounds slots).
 * Inside a call, fused dense gossip rounds other than the last two it may run do not store
 * their frontier rows (no later round reads them), so the delivery stream is available for
 * the last round a call ran, as after p2pg_step.                                          */
int p2pg_run(p2pg_engine* e, int32_t max_rounds, p2pg_round_stats* per_round,
             int32_t* n_rounds);
/* The first receipts of the most recent round, sorted by (peer, msg); parent = -1 at the
 * source.  Writes min(cap, count) records; *n_out = count (may exceed cap).
 * A round without first receipts has none (*n_out = 0).  P2PG_ERR_STATE if that round's
 * (or, for the parents, the previous round's) frontier was not kept -- not reachable through
 * p2pg_step / p2pg_run as specified above -- and for the round a snapshot was restored at
 * (p2pg_restore: the snapshot holds that round's frontier, not the one before it; the rounds
 * the restored engine runs report their deliveries as usual).                              */
int p2pg_get_new_deliveries(p2pg_engine* e, int64_t cap, int32_t* peer, int32_t* msg,
                            int32_t* hop, int32_t* parent, int64_t* n_out);
/* Every send of the most recent round -- the send_to_node calls its first receipts made
 * (node.py:114-120): flood, each connection but the one the receipt came from (all of them at
 * the origin, node.py:106-112); gossip, the k Philox picks -- as (sender, receiver, msg) records
 * sorted by (receiver, sender, msg), lost[i] = 1 if the send never arrives (churn drops it,
 * nodeconnection.py:123-126).  These are exactly the packets the next round's receivers hand to
 * node_message (nodeconnection.py:211-216), duplicates included; a p2pg_update_edges after this
 * call loses the ones on removed connections as well.  Reflects p2pg_drop_relays.  Writes
 * min(cap, count) records, *n_out = count.  P2PG_ERR_STATE after a p2pg_update_edges at this
 * round boundary or when the frontier (flood: and the one before it) was not kept.          */
int p2pg_get_sends(p2pg_engine* e, int64_t cap, int32_t* sender, int32_t* receiver, int32_t* msg,
                   uint8_t* lost, int64_t* n_out);
/* The app did not relay these first receipts of the most recent round (its node_message made no
 * send_to_nodes / send_to_node call for them, README.md:20): withdraw their sends before the
 * next round -- flood, their frontier bits; gossip, the round's pushes are redone without them.
 * Relay counters and the next round's `received` drop accordingly.  Each (peer[i], msg[i]) must
 * be a first receipt of that round, listed once (P2PG_ERR_ARG otherwise, nothing changed).
 * Read the round's deliveries first (they are its frontier bits).  Not on a vertex-partitioned
 * rank, not after a p2pg_update_edges at this boundary.                                      */
int p2pg_drop_relays(p2pg_engine* e, int64_t n, const int32_t* peer, const int32_t* msg);
/* Validation copies: seen [V][W] uint64 (W = ceil(M/64)); hop/parent [V][M] int32 need
 * P2PG_FLAG_RECORD (-1 = not delivered).  Any pointer may be NULL.                      */
int p2pg_read_planes(p2pg_engine* e, uint64_t* seen, int32_t* hop, int32_t* parent);
/* Word w of every peer's seen row (messages 64w .. 64w+63): out[V].  Full-size validation
 * without copying a whole plane (config 5: 51 GB at 100M peers x 4096 broadcasts).       */
int p2pg_read_seen_word(p2pg_engine* e, int32_t w, uint64_t* out);
/* Summed device time per kernel class since the last reset (needs P2PG_FLAG_TIMING):
 * 0 seed (origination), 1 flood pull, 2 gossip scatter by row atomics (sparse rounds),
 * 3 record (validation), 4 gossip update (consume row atomics), 5 gossip pull (consume edge
 * stores), 6 gossip scatter by edge stores (dense rounds), 7 gossip fused pull + scatter
 * (a dense round after a dense round).                                                  */
#define P2PG_KCLASS_N 8
int p2pg_kernel_times(p2pg_engine* e, double ms[P2PG_KCLASS_N], int64_t launches[P2PG_KCLASS_N]);
/* With P2PG_FLAG_TIMING: only launches of the classes in mask (bit i = class i; default all)
 * are bracketed by HIP events -- two event records per launch cost ~2.7 us of stream time each
 * (0.8 ms per config-4 broadcast), so a measurement can time its dominant kernel alone.
 * (Instrumentation; the reference has none -- its only counters are node.py:65-67.)       */
int p2pg_set_timed_classes(p2pg_engine* e, uint32_t mask);
/* ---- vertex-partitioned runs (one engine per GPU) ---------------------
 * The caller loads the rank's LOCAL graph: owned peers plus ghost peers (remote neighbours),
 * all numbered in ascending GLOBAL id order (so lowest-id tie-breaks are unchanged); ghosts
 * have empty rows.  gid[local] = global id (Philox keys, reported ids).  send_local = owned
 * boundary peers in the order the peers' ghost blocks expect them; recv_local = ghost peers
 * in the order the owners send them.  After each p2pg_step the caller moves rows between
 * ranks (e.g. RCCL all-to-all): plane 0 = frontier rows (pack from send_local, unpack into
 * recv_local, before the next flood step); plane 1 = gossip pushes addressed to ghosts (pack
 * from recv_local -- cleared locally --, unpack ORed into send_local).  Buffers are device
 * memory of n x W uint64 words.  Replaces the cross-host TCP fan-out of
 * NodeConnection.send (nodeconnection.py:107-160).                                      */
int p2pg_set_global_ids(p2pg_engine* e, const int32_t* gid);
/* Partitioned gossip, for hop / parent records and the delivery stream: a first receipt's
 * parent is the lowest-id neighbour whose Philox picks chose the receiver (node.py:334-338's
 * sender), and a GHOST neighbour's picks depend on its global degree and the
 * receiver's place in its global adjacency, which the rank-local graph does not hold:
 * ghost_deg[local] = global degree of each ghost (any value for owned peers), slot_pos[j] for
 * every local slot j = position of the slot's row owner in the neighbour's global ascending
 * adjacency when the neighbour is a ghost, else -1.  The ghosts' frontier rows must then also
 * travel each round (plane 0).  NULL, NULL removes them.                                   */
int p2pg_set_ghost_senders(p2pg_engine* e, const int32_t* ghost_deg, const int32_t* slot_pos);
int p2pg_set_exchange(p2pg_engine* e, int64_t n_send, const int32_t* send_local, int64_t n_recv,
                      const int32_t* recv_local);
int p2pg_exchange_pack(p2pg_engine* e, int32_t plane, void* dev_buf);
int p2pg_exchange_unpack(p2pg_engine* e, int32_t plane, const void* dev_buf);
/* Compacted exchange: only rows that carry something travel (plane 0: boundary peers with first
 * receipts this round; plane 1: ghosts that were pushed to), as records of 1 + W int64: the row's
 * index within the destination's list segment, then its W words.  The lists are cut into one
 * segment per rank (p2pg_set_exchange_segments: send / recv rows per rank, summing to the
 * set_exchange lists).  pack_live writes segment q's records from record send_off[q] of dev_buf
 * (capacity: the list length x (1 + W) int64) and returns the record count per destination in
 * counts[nseg] (host); unpack_live takes the records of all sources packed in source order and
 * their counts, and is asynchronous on the engine's stream.                               */
int p2pg_set_exchange_segments(p2pg_engine* e, int32_t nseg, const int64_t* send_counts,
                               const int64_t* recv_counts);
int p2pg_exchange_pack_live(p2pg_engine* e, int32_t plane, void* dev_buf, int64_t* counts);
/* Pack inside the round: from now on every p2pg_step / p2pg_step_end packs the live rows of
 * `plane` into dev_buf (same layout and capacity as pack_live) right after the round's kernels,
 * and the record counts come back together with the round counters -- one host
 * synchronisation per round instead of a second drain of the stream for the pack.  A following
 * p2pg_exchange_pack_live(e, plane, dev_buf, counts) then only returns those counts.  NULL turns
 * it off.  (Replaces, like pack_live, the cross-host fan-out of NodeConnection.send,
 * nodeconnection.py:107-160.)                                                              */
int p2pg_set_exchange_buffer(p2pg_engine* e, int32_t plane, void* dev_buf);
int p2pg_exchange_unpack_live(p2pg_engine* e, int32_t plane, const void* dev_buf, const int64_t* counts);
/* A round in two calls, so a vertex-partitioned rank overlaps the exchange of the last round's
 * rows with work: step_begin launches the pull / update of the peers with no ghost neighbour
 * (they need none of the exchanged rows) and returns at once; step_end runs the rest of the
 * round once the rows are unpacked (= p2pg_step).  p2pg_step alone does both.  Between the
 * two, snapshot / restore / update_edges / set_exchange / exchange packing are refused
 * (P2PG_ERR_STATE): the round is half done.                                                */
int p2pg_step_begin(p2pg_engine* e);
int p2pg_step_end(p2pg_engine* e, p2pg_round_stats* out);
/* ---- dynamic topology --------------------------------------------
 * Connection changes between rounds: n_add pairs to connect (Node.connect_with_node,
 * node.py:122-176) and n_del pairs to disconnect (Node.disconnect_with_node, node.py:178-189,
 * then node_disconnected on both ends, node.py:307-319), as 2*n peer ids (a0, b0, a1, b1..).
 * Connecting an existing pair, disconnecting a missing one, self connections and pairs listed
 * twice are errors (P2PG_ERR_ARG; the reference refuses them with a debug print).  Messages
 * sent in the last round and still in flight on a removed connection are lost (a stopped
 * NodeConnection drops its unread buffer, nodeconnection.py:192-228); the others arrive next
 * round; every send from the next round on uses the new connections.  One update per round
 * boundary; not on a vertex-partitioned rank.                                              */
int p2pg_update_edges(p2pg_engine* e, int64_t n_add, const int32_t* add, int64_t n_del,
                      const int32_t* del);
/* ---- snapshot / resume (the reference has no checkpointing) --------
 * Between rounds, the run state (round, seen sets, saturation, the last round's first
 * receipts, messages in flight, hop/parent planes in record mode) is written to a caller
 * buffer of p2pg_snapshot_size bytes, and read back by p2pg_restore into an engine with the
 * same configuration, graph and sources (checked: P2PG_ERR_STATE otherwise), which then
 * continues bit-identically.  Not between a topology update and the next round.           */
int p2pg_snapshot_size(p2pg_engine* e, int64_t* bytes);
int p2pg_snapshot(p2pg_engine* e, void* buf, int64_t cap);
int p2pg_restore(p2pg_engine* e, const void* buf, int64_t size);
/* Launch on this hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL =
 * the engine's own stream.                                                              */
int p2pg_set_stream(p2pg_engine* e, void* hip_stream);
/* Device-side Philox KAT: evaluates philox4x32_10 on n counters with one key.          */
int p2pg_device_philox(p2pg_engine* e, int32_t n, const uint32_t* ctr, const uint32_t key[2],
                       uint32_t* out);
const char* p2pg_last_error(const p2pg_engine* e);
const char* p2pg_global_error(void);
void p2pg_destroy(p2pg_engine* e);

#ifdef __cplusplus
}
#endif
#endif /* P2PGPU_H */
