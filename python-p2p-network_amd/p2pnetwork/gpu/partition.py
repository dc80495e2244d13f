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


class VertexPartition:
    """Contiguous peer ranges balanced by directed-connection count; rank-local CSR."""

    def __init__(self, graph, world, rank):
        if not 0 <= rank < world:
            raise ValueError("rank out of range")
        self.world, self.rank = world, rank
        V = graph.V
        rp = graph.rowptr
        nnz = int(rp[-1])
        # bounds[q] = first peer of rank q (edge-balanced), bounds[world] = V
        targets = (np.arange(1, world, dtype=np.float64) * nnz / world)
        cuts = np.searchsorted(rp[:-1], targets, side="left")
        self.bounds = np.concatenate([[0], np.maximum.accumulate(cuts), [V]]).astype(np.int64)
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
        owned_local = np.searchsorted(self.gid, np.arange(lo, hi))
        self.owned_local = owned_local.astype(np.int64)
        # local CSR: owned rows mapped (monotone map keeps rows ascending), ghost rows empty
        deg_local = np.zeros(self.V_local, dtype=np.int64)
        deg_local[owned_local] = np.diff(rp[lo:hi + 1])
        self.rowptr = np.concatenate([[0], np.cumsum(deg_local)]).astype(np.int64)
        self.colidx = np.searchsorted(self.gid, nb).astype(np.int32)
        # exchange lists, peer by peer, each sorted by global id
        owner = self.owner(ghosts)
        self.recv_counts = np.bincount(owner, minlength=world).astype(np.int64)
        self.recv_counts[rank] = 0
        self.recv_local = np.searchsorted(self.gid, ghosts).astype(np.int32)  # ghosts by owner
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
        self.send_local = np.searchsorted(self.gid, send).astype(np.int32)

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


def live_rows(send, send_counts, W):
    """Compaction of an exchange buffer: (mask, rows, counts) = a uint8 flag per row (row has a
    non-zero word), the live rows in order, and the live-row count per destination segment.
    Dead rows carry nothing: a flood row of an inactive boundary peer (the receiver's pull has
    already cleared the ghost's activity bit for the round) or a gossip ghost nobody pushed to."""
    import torch
    n = int(np.sum(send_counts))
    rows = send[:n * W].view(n, W)
    live = (rows != 0).any(dim=1)
    bounds = np.concatenate([[0], np.cumsum(send_counts)]).astype(np.int64)
    per = [live[int(a):int(b)].sum() for a, b in zip(bounds[:-1], bounds[1:])]
    counts = torch.stack(per).cpu().numpy().astype(np.int64) if per else np.zeros(0, np.int64)
    return live.to(torch.uint8), rows[live].reshape(-1), counts


def expand_rows(mask, rows, W):
    """Inverse of live_rows on the receiving side: full rows, zeros where the flag is 0."""
    import torch
    full = torch.zeros((mask.numel(), W), dtype=rows.dtype, device=rows.device)
    full[mask.to(torch.bool)] = rows.view(-1, W)
    return full.view(-1)


class TorchTransport:
    """All-to-all and sum-reduce over a torch.distributed process group.  With the nccl
    backend (RCCL on ROCm) the rows move device-to-device over xGMI; with gloo they are
    staged through host memory (CPU tests, or two ranks sharing one GPU).

    Rows go compacted (``sparse``, default): one byte per boundary row says whether the row
    travels, and only rows with a non-zero word do -- outside the peak rounds most boundary
    peers are inactive, and the all-to-all moves 512 B per row otherwise."""

    def __init__(self, device=None, group=None, sparse=True):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.backend = dist.get_backend(group)
        self.device = device
        self.sparse = sparse
        self.rows_total = 0  # boundary rows offered / actually sent (exchange volume)
        self.rows_sent = 0

    def _a2a(self, recv, send, outs, ins):
        torch, dist = self.torch, self.dist
        if self.backend == "nccl":
            dist.all_to_all_single(recv, send, outs, ins, group=self.group)
            torch.cuda.synchronize(send.device)
            return recv
        r = recv.cpu()
        dist.all_to_all_single(r, send.cpu(), outs, ins, group=self.group)
        return r.to(send.device)

    def alltoall_rows(self, send, send_counts, recv_counts, W):
        """send: tensor [sum(send_counts) * W] int64 (on self.device); returns the recv tensor
        (full rows, in the receiver's list order)."""
        torch = self.torch
        n_out, n_in = int(sum(send_counts)), int(sum(recv_counts))
        self.rows_total += n_out
        if not self.sparse:
            self.rows_sent += n_out
            recv = torch.empty(n_in * W, dtype=torch.int64, device=send.device)
            return self._a2a(recv, send[:n_out * W], [int(c) * W for c in recv_counts],
                             [int(c) * W for c in send_counts])
        mask, rows, live = live_rows(send, send_counts, W)
        self.rows_sent += int(live.sum())
        dev = send.device
        cnt = torch.as_tensor(live, dtype=torch.int64, device=dev)
        got = self._a2a(torch.empty(len(recv_counts), dtype=torch.int64, device=dev), cnt,
                        [1] * len(recv_counts), [1] * len(send_counts)).cpu().numpy()
        rmask = self._a2a(torch.empty(n_in, dtype=torch.uint8, device=dev), mask,
                          [int(c) for c in recv_counts], [int(c) for c in send_counts])
        rrows = self._a2a(torch.empty(int(got.sum()) * W, dtype=torch.int64, device=dev), rows,
                          [int(c) * W for c in got], [int(c) * W for c in live])
        return expand_rows(rmask, rrows, W)

    def allreduce_sum(self, values):
        torch, dist = self.torch, self.dist
        dev = self.device if self.backend == "nccl" else "cpu"
        t = torch.tensor(np.asarray(values, dtype=np.int64), device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t.cpu().numpy()


class PartitionedNetwork:
    """The relay of ``GraphNetwork`` on one rank of a vertex-partitioned multi-GPU job."""

    def __init__(self, graph, world, rank, transport, mode="flood", fanout=3, gossip_seed=0x5EED,
                 churn_threshold_value=0, churn_seed=0xC0FFEE, record=False, timing=False,
                 device=0, engine_factory=None):
        if record and mode == "gossip" and world > 1:
            # a gossip parent check needs the REMOTE sender's degree and adjacency order
            raise NotImplementedError("record=True for partitioned gossip: record on one GPU")
        self.graph, self.world, self.rank, self.transport = graph, world, rank, transport
        self.mode, self.fanout = mode, fanout
        self.part = VertexPartition(graph, world, rank)
        make = engine_factory or GraphNetwork
        self.net = make(self.part.local_graph(), mode=mode, fanout=fanout, gossip_seed=gossip_seed,
                        churn_threshold_value=churn_threshold_value, churn_seed=churn_seed,
                        record=record, timing=timing, device=device, autostop=False,
                        local_graph=True)
        self.net.set_global_ids(self.part.gid)
        self.net.set_exchange(self.part.send_local, self.part.recv_local)
        self.rounds = []        # global counters (summed over ranks)
        self.local_rounds = []  # this rank's engine counters (its owned peers' work)
        self.exchange_s = 0.0   # host wall time spent in the row exchange since reset
        self.sources = None

    @property
    def M(self):
        return 0 if self.sources is None else len(self.sources)

    def broadcast(self, sources):
        self.sources = np.asarray(sources, dtype=np.int64)
        self.net.broadcast(self.part.local_sources(self.sources))
        self.rounds, self.local_rounds, self.exchange_s = [], [], 0.0

    def reset(self):
        self.net.reset()
        self.rounds, self.local_rounds, self.exchange_s = [], [], 0.0

    def _round0_stats(self):
        """Origination counted once, globally (every rank seeds origins it holds as ghosts)."""
        deg = self.graph.degree()
        src = self.sources
        W = (self.M + 63) // 64
        per = np.minimum(deg[src], self.fanout) if self.mode == "gossip" else deg[src]
        vs = np.unique(src)
        words = np.unique(src * W + np.arange(self.M) // 64)
        return RoundStats(round=0, active=1, new_deliveries=self.M, relays=int(per.sum()),
                          active_vertices=len(vs), active_words=len(words),
                          wedges=int(deg[words // W].sum()), deg_active=int(deg[vs].sum()),
                          scatter_words=0, touched_words=0)

    @staticmethod
    def _ready(t):
        """The transport builds the received rows with torch ops on torch's current stream; the
        engine unpacks on its own stream, so wait for them first (nothing else orders them)."""
        if getattr(t, "is_cuda", False):
            import torch
            torch.cuda.current_stream(t.device).synchronize()
        return t

    def _exchange(self):
        if self.world == 1:
            return
        W = (self.M + 63) // 64
        p = self.part
        if self.mode == "flood":   # frontier rows: owner -> ghost holders
            send = self.net.alloc_exchange(int(p.send_counts.sum()) * W)
            self.net.exchange_pack(0, send)
            recv = self.transport.alltoall_rows(send, p.send_counts, p.recv_counts, W)
            self.net.exchange_unpack(0, self._ready(recv))
        else:                      # gossip pushes: ghost holder -> owner
            send = self.net.alloc_exchange(int(p.recv_counts.sum()) * W)
            self.net.exchange_pack(1, send)
            recv = self.transport.alltoall_rows(send, p.recv_counts, p.send_counts, W)
            self.net.exchange_unpack(1, self._ready(recv))

    def step(self):
        st = self.net.step()
        self.local_rounds.append(st)
        t0 = time.perf_counter()
        self._exchange()
        self.exchange_s += time.perf_counter() - t0
        if st.round == 0:
            g = self._round0_stats()
            # scatter words of round 0 are real local work (gossip): sum them
            sw = int(self.transport.allreduce_sum([st.scatter_words])[0]) if self.world > 1 else st.scatter_words
            g.scatter_words = sw
        else:
            vals = [getattr(st, f) for f in STAT_FIELDS[2:]]
            tot = self.transport.allreduce_sum(vals) if self.world > 1 else np.asarray(vals)
            g = RoundStats(st.round, int(tot[0] > 0), *[int(x) for x in tot])
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

    def owned_planes(self):
        """(global ids, seen rows) of the peers this rank owns."""
        s = self.net.seen_plane()
        return self.part.gid[self.part.owned_local], s[self.part.owned_local]

    def owned_hop_parent(self):
        hop, par = self.net.hop_parent()
        return self.part.gid[self.part.owned_local], hop[self.part.owned_local], par[self.part.owned_local]

    def close(self):
        self.net.close()
