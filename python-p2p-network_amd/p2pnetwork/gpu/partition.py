"""Vertex-partitioned relay over several GPUs (one process per GPU).

In p2pnetwork, peers on different hosts relay to each other over TCP
(``NodeConnection.send``, p2pnetwork/nodeconnection.py:107-160).  Here the peer graph is split
into contiguous peer-id ranges, balanced by connection count; each rank runs the engine on its
range plus *ghost* copies of the remote neighbours of its peers.  After every round the ranks
exchange rows with one all-to-all (RCCL over xGMI via torch.distributed on GPUs, gloo in CPU
tests):

* flood: the frontier rows of boundary peers go owner -> ranks holding them as ghosts, where the
  next round's pull reads them like local rows;
* gossip: pushes addressed to ghosts go ghost -> owner, ORed into the owner's push rows.

Only rows that carry something travel (records packed on the device), and the peers without a
ghost neighbour run the next round while the records are in flight.

Local ids follow global id order (ghosts interleaved), so every ascending-id rule (the
lowest-id sender tie-break, gossip's sorted candidate list) is the same as on one GPU, and the
Philox keys of gossip and churn use global ids: results are bit-identical to a single-engine
run.  A dummy, unconnected local peer (global id V) absorbs broadcasts whose origin is neither
owned nor a ghost here.
"""
import time

import numpy as np

from .graph import PeerGraph
from .network import GraphNetwork, RoundStats, STAT_FIELDS

MAX_RANKS = 16  # exchange segments per engine (P2PG_MAX_RANKS, csrc/internal.h)


class VertexPartition:
    """Contiguous peer ranges balanced by directed-connection count; rank-local CSR."""

    def __init__(self, graph, world, rank):
        if not 0 <= rank < world:
            raise ValueError("rank out of range")
        self.world, self.rank = world, rank
        V = graph.V
        rp = graph.rowptr
        self.bounds = self.ranges(graph, world)
        lo, hi = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.lo, self.hi = lo, hi
        nb = graph.colidx[rp[lo]:rp[hi]].astype(np.int64)
        remote = nb[(nb < lo) | (nb >= hi)]
        ghosts = np.unique(remote)
        # local ids: owned range and ghosts merged in global order, plus a dummy sink (gid V)
        gid = np.union1d(np.arange(lo, hi, dtype=np.int64), ghosts)
        self.gid = np.concatenate([gid, [V]]).astype(np.int32)
        self.V_local = len(self.gid)
        self.dummy = self.V_local - 1
        # global -> local id of every held peer by one dense map (a binary search per slot took
        # ~2 minutes per rank at config 5's 100M peers; the map is 4 B per global peer)
        loc = np.empty(V, dtype=np.int32)
        loc[gid] = np.arange(len(gid), dtype=np.int32)
        owned_local = loc[lo:hi].astype(np.int64)
        self.owned_local = owned_local
        # local CSR: owned rows mapped (monotone map keeps rows ascending), ghost rows empty
        deg_local = np.zeros(self.V_local, dtype=np.int64)
        deg_local[owned_local] = np.diff(rp[lo:hi + 1])
        self.rowptr = np.concatenate([[0], np.cumsum(deg_local)]).astype(np.int64)
        self.colidx = loc[nb]
        # exchange lists, peer by peer, each sorted by global id
        owner = self.owner(ghosts)
        self.recv_counts = np.bincount(owner, minlength=world).astype(np.int64)
        self.recv_counts[rank] = 0
        self.recv_local = loc[ghosts]  # ghosts by owner
        rows = np.repeat(np.arange(lo, hi, dtype=np.int64), np.diff(rp[lo:hi + 1]))
        is_remote = (nb < lo) | (nb >= hi)
        pairs_peer = self.owner(nb[is_remote])
        pairs_src = rows[is_remote]
        send, counts = [], np.zeros(world, dtype=np.int64)
        for p in range(world):
            if p == rank:
                continue
            s = np.unique(pairs_src[pairs_peer == p])
            counts[p] = len(s)
            send.append(s)
        send = np.concatenate(send) if send else np.zeros(0, dtype=np.int64)
        self.send_counts = counts
        self.send_local = loc[send]

    @staticmethod
    def ranges(graph, world):
        """bounds[q] = first peer of rank q (contiguous ranges balanced by connection count),
        bounds[world] = V."""
        rp = graph.rowptr
        nnz = int(rp[-1])
        targets = (np.arange(1, world, dtype=np.float64) * nnz / world)
        cuts = np.searchsorted(rp[:-1], targets, side="left")
        return np.concatenate([[0], np.maximum.accumulate(cuts), [graph.V]]).astype(np.int64)

    def ghost_senders(self, graph):
        """(ghost_deg [V_local], slot_pos [local slots]) for p2pg_set_ghost_senders: a ghost's
        global degree, and for every local slot whose neighbour is a ghost the row owner's
        position in that ghost's global ascending adjacency (-1 for a local neighbour) -- what
        replaying a remote sender's gossip picks needs (hop / parent records, deliveries)."""
        rp, ci = graph.rowptr, graph.colidx
        V = graph.V
        gid = self.gid[:-1].astype(np.int64)            # without the dummy sink
        ghost_deg = np.zeros(self.V_local, dtype=np.int32)
        ghost_deg[:-1] = (rp[gid + 1] - rp[gid]).astype(np.int32)
        nb = gid[self.colidx.astype(np.int64)]          # global neighbour of each local slot
        rows = np.repeat(gid, np.diff(self.rowptr)[:-1])  # row owner of each slot (dummy: none)
        remote = (nb < self.lo) | (nb >= self.hi)
        pos = np.full(len(nb), -1, dtype=np.int32)
        if remote.any():
            us, vs = nb[remote], rows[remote]
            # the ghosts' global rows, concatenated in ascending (ghost, neighbour) key order
            ghosts = np.unique(us)
            starts, ends = rp[ghosts], rp[ghosts + 1]
            lens = ends - starts
            off = np.concatenate([[0], np.cumsum(lens)])
            idx = np.repeat(starts - off[:-1], lens) + np.arange(off[-1])
            keys = np.repeat(ghosts, lens) * V + ci[idx].astype(np.int64)
            at = np.searchsorted(keys, us * V + vs)
            assert np.array_equal(keys[at], us * V + vs), "asymmetric adjacency"
            pos[remote] = (at - off[np.searchsorted(ghosts, us)]).astype(np.int32)
        return ghost_deg, pos

    def owner(self, g):
        return (np.searchsorted(self.bounds, np.asarray(g), side="right") - 1).astype(np.int64)

    def local_graph(self):
        return PeerGraph(self.rowptr, self.colidx, validate=False)

    def local_sources(self, src):
        """Global origins -> local ids (dummy sink where the origin is not held here)."""
        src = np.asarray(src, dtype=np.int64)
        pos = np.searchsorted(self.gid[:-1], src)
        pos = np.minimum(pos, len(self.gid) - 2)
        held = self.gid[pos] == src
        return np.where(held, pos, self.dummy).astype(np.int32)


def host_group_for(group=None):
    """A gloo group with the ranks of ``group`` (None = the default group), for the host-side
    count all-gather next to an RCCL group.  Collective over the default group: call it on
    every rank of the job."""
    import torch.distributed as dist
    ranks = list(range(dist.get_world_size())) if group is None else dist.get_process_group_ranks(group)
    return dist.new_group(ranks=ranks, backend="gloo")


class TorchTransport:
    """The two collectives of a partitioned round over a torch.distributed process group.
    With the nccl backend (RCCL on ROCm) records move device-to-device over xGMI; with gloo
    they are staged through host memory (CPU tests, or ranks sharing one GPU).

    * ``exchange_counts(vec)``: all-gather of one small int64 vector per rank (each rank's
      record count per destination + its round counters) -> [world, len].  The vector is on the
      host already (the pack reads its counts back), so it goes over a host (gloo) group: no
      device round trip, no stream synchronisation;
    * ``exchange_records(...)``: ONE all-to-all of the packed records per round
      (``all_to_all_single`` with per-rank split sizes = RCCL's all-to-all-v over xGMI): each
      rank's records for rank q, compacted in destination order, land in rank q's receive
      buffer in source order -- exactly the live rows each peer rank needs;
    * ``engine_stream()``: the stream the rank's engine should launch on (device runs), so
      that the collective's completion is ordered before the unpack by a stream wait, not a
      host sync."""

    def __init__(self, device=None, group=None, host_group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.backend = dist.get_backend(group)
        self.device = device
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        # counts travel host-side; with RCCL that needs a gloo group next to the nccl one.
        # Pass it in (host_group_for) when `group` is a subgroup: creating a group is collective
        # over the DEFAULT group, so every rank of the job must make that call, not only the
        # ranks that build a transport.
        if self.backend == "gloo":
            self.host_group = group
        elif host_group is not None:
            self.host_group = host_group
        elif group is None:
            self.host_group = host_group_for(None)
        else:
            raise ValueError("TorchTransport over an RCCL subgroup: pass host_group="
                             "host_group_for(group), created by every rank of the job")
        self.rows_total = 0  # boundary rows offered / actually sent (exchange volume)
        self.rows_sent = 0
        self.collectives = 0  # all-to-alls issued

    def engine_stream(self):
        if self.device is None or not str(self.device).startswith("cuda"):
            return None
        return self.torch.cuda.Stream(device=self.device)

    def exchange_counts(self, vec):
        torch, dist = self.torch, self.dist
        t = torch.as_tensor(np.asarray(vec, dtype=np.int64))
        out = torch.empty(self.world * t.numel(), dtype=torch.int64)
        dist.all_gather_into_tensor(out, t, group=self.host_group)
        return out.numpy().reshape(self.world, -1)

    def _all_to_all(self, out, inp, out_splits, in_splits):
        """The collective: all_to_all_single over the transport's group (RCCL on device tensors:
        one all-to-all-v, issued on torch's current stream)."""
        self.dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def exchange_records(self, send_buf, send_off, send_cnt, recv_buf, recv_cnt, R):
        """send_buf: records to rank q at record send_off[q], send_cnt[q] of them; recv_buf:
        the records from every source rank, packed in source order (R int64 per record).  Every
        rank calls it every round (a collective), also with nothing to move."""
        torch = self.torch
        in_splits = [int(c) * R for c in send_cnt]
        out_splits = [int(c) * R for c in recv_cnt]
        segs = [send_buf[int(send_off[q]) * R:int(send_off[q]) * R + in_splits[q]]
                for q in range(self.world) if in_splits[q]]
        x = torch.cat(segs) if len(segs) > 1 else segs[0] if segs else send_buf[:0]
        y = recv_buf[:sum(out_splits)]
        stage = self.backend != "nccl" and send_buf.is_cuda  # gloo moves host tensors only
        if stage:
            x, land = x.cpu(), torch.empty(y.shape, dtype=y.dtype)
            self._all_to_all(land, x, out_splits, in_splits)
            y.copy_(land)
        else:
            self._all_to_all(y, x, out_splits, in_splits)
        self.collectives += 1


class PartitionedNetwork:
    """The relay of ``GraphNetwork`` on one rank of a vertex-partitioned multi-GPU job.

    Per round r (``step``): finish round r on this rank (``p2pg_step_end``), pack its live
    boundary rows on the device (``p2pg_exchange_pack_live``: one record per row that carries
    something, counted per destination), one all-gather of (record counts, round counters),
    then -- while the grouped sends / receives of the records are in flight -- the interior
    peers of round r+1 (no ghost neighbour) already run (``p2pg_step_begin``); the records are
    unpacked (``p2pg_exchange_unpack_live``) before the border peers of round r+1 run."""

    def __init__(self, graph, world, rank, transport, mode="flood", fanout=3, gossip_seed=0x5EED,
                 churn_threshold_value=0, churn_seed=0xC0FFEE, record=False, timing=False,
                 device=0, engine_factory=None, overlap=True, deliveries=False, msg_id_base=0):
        if not 1 <= world <= MAX_RANKS:
            raise ValueError(f"vertex partition over {world} ranks: the exchange supports 1..{MAX_RANKS}")
        self.world, self.rank, self.transport = world, rank, transport
        # partitioned gossip with hop / parent records or the per-round delivery stream: a
        # parent is the lowest-id neighbour whose picks chose the receiver (node.py:334-338's
        # sender), and for a ghost sender the rank needs its frontier rows (plane 0 travels
        # too, owner -> ghost holders) and its global degree / adjacency order
        self._senders = mode == "gossip" and world > 1 and (record or deliveries)
        self._deliv = deliveries
        self._last_deliv = None
        self.deg = graph.degree().astype(np.int32)  # global degrees (round-0 counters); the
        # global graph itself is not kept: the engine holds only the rank-local CSR
        self.mode, self.fanout = mode, fanout
        self._plane = 0 if mode == "flood" else 1  # rows that travel: frontier / ghost pushes
        self.overlap = overlap
        self.part = VertexPartition(graph, world, rank)
        make = engine_factory or GraphNetwork
        # msg_id_base: this job's broadcasts are messages msg_id_base.. of a larger set (a message
        # split on top of the vertex partition: each group of ranks runs its own share)
        extra = {"msg_id_base": msg_id_base} if msg_id_base else {}
        self.net = make(self.part.local_graph(), mode=mode, fanout=fanout, gossip_seed=gossip_seed,
                        churn_threshold_value=churn_threshold_value, churn_seed=churn_seed,
                        record=record, timing=timing, device=device, autostop=False,
                        local_graph=True, **extra)
        # device runs: the engine launches on a torch stream of its own, so the receives (torch's
        # current stream, which RCCL orders after its transfers) are ordered before the unpack by
        # a stream wait (_ready), and the next round's interior peers still overlap the transfers
        st = getattr(transport, "engine_stream", None)
        self._stream = st() if st is not None else None
        if self._stream is not None:
            self.net.set_stream(self._stream.cuda_stream)
        self.net.set_global_ids(self.part.gid)
        self.net.set_exchange(self.part.send_local, self.part.recv_local)
        self.net.set_exchange_segments(self.part.send_counts, self.part.recv_counts)
        if self._senders:
            self.net.set_ghost_senders(*self.part.ghost_senders(graph))
        self.rounds = []        # global counters (summed over ranks)
        self.local_rounds = []  # this rank's engine counters (its owned peers' work)
        self.exchange_s = 0.0   # host wall time spent in the row exchange since reset
        self.sources = None
        self._begun = False
        self._bufs = None

    @property
    def M(self):
        return 0 if self.sources is None else len(self.sources)

    def broadcast(self, sources):
        self.sources = np.asarray(sources, dtype=np.int64)
        self.net.broadcast(self.part.local_sources(self.sources))
        self.rounds, self.local_rounds, self.exchange_s = [], [], 0.0
        self._begun = False
        W = (self.M + 63) // 64
        rows = max(len(self.part.send_local), len(self.part.recv_local), 1)
        self._bufs = (self.net.alloc_exchange(rows * (1 + W)), self.net.alloc_exchange(rows * (1 + W)))
        self._fbufs = ((self.net.alloc_exchange(rows * (1 + W)), self.net.alloc_exchange(rows * (1 + W)))
                       if self._senders else None)
        if self.world > 1 and hasattr(self.net, "set_exchange_buffer"):
            # the round packs its live rows itself: their counts arrive with the round counters,
            # so exchange_pack_live below costs no second stream drain before the sends
            self.net.set_exchange_buffer(self._plane, self._bufs[0])

    def reset(self):
        self.net.reset()
        self.rounds, self.local_rounds, self.exchange_s = [], [], 0.0
        self._begun = False

    def _round0_stats(self):
        """Origination counted once, globally (every rank seeds origins it holds as ghosts)."""
        deg = self.deg.astype(np.int64)
        src = self.sources
        W = (self.M + 63) // 64
        per = np.minimum(deg[src], self.fanout) if self.mode == "gossip" else deg[src]
        vs = np.unique(src)
        words = np.unique(src * W + np.arange(self.M) // 64)
        return RoundStats(round=0, active=1, new_deliveries=self.M, relays=int(per.sum()),
                          active_vertices=len(vs), active_words=len(words),
                          wedges=int(deg[words // W].sum()), deg_active=int(deg[vs].sum()),
                          scatter_words=0, touched_words=0)

    def _ready(self, t):
        """Records received with torch ops / RCCL are ordered on torch's current stream; the
        engine unpacks on its own stream, which waits for them on the device (no host sync)."""
        if getattr(t, "is_cuda", False):
            import torch
            if self._stream is None:  # an engine on a stream torch does not know: host sync
                torch.cuda.current_stream(t.device).synchronize()
            else:
                self._stream.wait_stream(torch.cuda.current_stream(t.device))
        return t

    def _send_rows(self, plane):
        p = self.part
        # plane 0: frontier rows owner -> ghost holders; plane 1: pushes ghost -> owner
        return p.send_counts if plane == 0 else p.recv_counts

    def _senders_frontier(self):
        """Gossip records / deliveries: the boundary peers' frontier rows of this round to the
        ranks holding them as ghosts (plane 0), before the next round begins."""
        R = 1 + (self.M + 63) // 64
        send_off = np.concatenate([[0], np.cumsum(self._send_rows(0))]).astype(np.int64)
        sbuf, rbuf = self._fbufs
        counts = np.asarray(self.net.exchange_pack_live(0, sbuf), dtype=np.int64)
        recv_cnt = self.transport.exchange_counts(counts)[:, self.rank].copy()
        self.transport.exchange_records(sbuf, send_off, counts, rbuf, recv_cnt, R)
        self.net.exchange_unpack_live(0, self._ready(rbuf), recv_cnt)

    def step(self):
        if not self._begun:
            self.net.step_begin()
        st = self.net.step_end()
        self._begun = False
        self.local_rounds.append(st)
        if self._deliv:
            # before the next round begins (its interior peers overwrite the frontier plane the
            # parents of this round's receipts are read from)
            self._last_deliv = self._owned_deliveries()
        vals = np.asarray([getattr(st, f) for f in STAT_FIELDS[2:]], dtype=np.int64)
        if self.world == 1:
            tot = vals
        else:
            t0 = time.perf_counter()
            W = (self.M + 63) // 64
            R = 1 + W
            plane = self._plane
            send_rows = self._send_rows(plane)
            send_off = np.concatenate([[0], np.cumsum(send_rows)]).astype(np.int64)
            sbuf, rbuf = self._bufs
            if self._senders:
                self._senders_frontier()
            counts = np.asarray(self.net.exchange_pack_live(plane, sbuf), dtype=np.int64)
            allv = self.transport.exchange_counts(np.concatenate([counts, vals]))
            recv_cnt = allv[:, self.rank].copy()
            tot = allv[:, self.world:].sum(axis=0)
            self.transport.rows_total += int(send_rows.sum())
            self.transport.rows_sent += int(counts.sum())
            if self.overlap and tot[0] > 0:
                self.net.step_begin()  # round r+1's interior peers, while the records travel
                self._begun = True
            self.transport.exchange_records(sbuf, send_off, counts, rbuf, recv_cnt, R)
            self.net.exchange_unpack_live(plane, self._ready(rbuf), recv_cnt)
            self.exchange_s += time.perf_counter() - t0
        if st.round == 0:
            g = self._round0_stats()
            g.scatter_words = int(tot[STAT_FIELDS[2:].index("scatter_words")])
        else:
            g = RoundStats(st.round, int(tot[0] > 0), *[int(x) for x in tot],
                           received_exact=st.received_exact)
        self.rounds.append(g)
        return g

    def run(self, max_rounds=1 << 20):
        out = []
        while len(out) < max_rounds:
            st = self.step()
            out.append(st)
            if not st.new_deliveries:
                break
        return out

    @property
    def message_count_send(self):
        return sum(r.relays for r in self.rounds)

    def kernel_times(self):
        return self.net.kernel_times()

    def set_timed_classes(self, classes=None):
        self.net.set_timed_classes(classes)

    def owned_planes(self):
        """(global ids, seen rows) of the peers this rank owns."""
        s = self.net.seen_plane()
        return self.part.gid[self.part.owned_local], s[self.part.owned_local]

    def deliveries(self):
        """The first receipts of the last round at the peers this rank owns, as Deliveries with
        global peer / parent ids (sorted by (peer, msg)): this rank's share of the batched
        node_message hook (node.py:334-338).  Needs PartitionedNetwork(deliveries=True): they are
        taken inside step(), before the next round's interior peers start."""
        if not self._deliv:
            raise RuntimeError("partitioned deliveries need PartitionedNetwork(deliveries=True)")
        return self._last_deliv

    def _owned_deliveries(self):
        from .network import Deliveries
        # the local stream also holds the ghosts' receipts (their rows arrived as plane 0)
        n = self.net.deliveries_count()
        d = self.net.deliveries(cap=n)
        own = (d.peer >= self.part.lo) & (d.peer < self.part.hi)
        return Deliveries(d.peer[own], d.msg[own], d.hop[own], d.parent[own])

    def owned_hop_parent(self):
        hop, par = self.net.hop_parent()
        return self.part.gid[self.part.owned_local], hop[self.part.owned_local], par[self.part.owned_local]

    def close(self):
        self.net.close()
