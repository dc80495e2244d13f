"""Test-only NumPy stand-in for one rank's engine in a vertex-partitioned run (CPU tests of
p2pnetwork.gpu.partition with the gloo backend, and of compat mode on one "rank").  It restates, on the rank-local graph with
ghost rows, exactly the contract of the C-ABI's partition entry points (include/p2pgpu.h):
frontier rows valid only with their A bit, ghost rows filled by unpack, pushes to ghosts moved
by pack/unpack, Philox keys on global ids.  Uses the oracle's Philox (tests may)."""
import numpy as np

from oracle import philox
from p2pnetwork.gpu.network import RoundStats


def _words(b):
    """bool [n, M] -> uint64 [n, W]"""
    n, M = b.shape
    W = (M + 63) // 64
    pad = np.zeros((n, W * 64), dtype=bool)
    pad[:, :M] = b
    return np.packbits(pad.reshape(n, W, 64), axis=2, bitorder="little").reshape(n, W * 8).view(np.uint64)


def _bits(w, M):
    n = w.shape[0]
    if n == 0:
        return np.zeros((0, M), dtype=bool)
    return np.unpackbits(w.view(np.uint8).reshape(n, -1), axis=1, bitorder="little")[:, :M].astype(bool)


class MockEngine:
    def __init__(self, graph, mode="flood", fanout=3, gossip_seed=0, churn_threshold_value=0,
                 churn_seed=0, record=False, timing=False, device=0, autostop=True, local_graph=False,
                 count_received=False):
        self.g, self.mode, self.k = graph, mode, fanout
        self.gseed, self.thr, self.cseed = gossip_seed, churn_threshold_value, churn_seed
        self.V = graph.V
        self.deg = graph.degree()
        self.rows = np.repeat(np.arange(self.V), self.deg)
        self.gid = np.arange(self.V)

    def set_global_ids(self, gid):
        self.gid = np.asarray(gid, dtype=np.int64)

    def set_exchange(self, send_local, recv_local):
        self.send, self.recv = np.asarray(send_local), np.asarray(recv_local)

    def set_exchange_segments(self, send_counts, recv_counts):
        self.send_off = np.concatenate([[0], np.cumsum(send_counts)]).astype(np.int64)
        self.recv_off = np.concatenate([[0], np.cumsum(recv_counts)]).astype(np.int64)

    def step_begin(self):
        pass

    def step_end(self):
        return self.step()

    def alloc_exchange(self, n_words):
        import torch
        return torch.zeros(max(int(n_words), 1), dtype=torch.int64)

    def broadcast(self, src):
        self.src = np.asarray(src, dtype=np.int64)
        self.M = len(self.src)
        self.reset()

    def reset(self):
        V, M = self.V, self.M
        self.seen = np.zeros((V, M), bool)
        self.F = np.zeros((V, M), bool)
        self.next = np.zeros((V, M), bool)
        self.cand = np.full((V, M), np.iinfo(np.int64).max)
        self.hop = np.full((V, M), -1, np.int32)
        self.par = np.full((V, M), -1, np.int32)
        self.round = 0

    def _stats(self, new, per_bit, scatter=0):
        W = (self.M + 63) // 64
        words = _words(new) != 0
        pv = new.sum(1)
        act = pv > 0
        return RoundStats(self.round, int(pv.sum() > 0), int(pv.sum()), int((pv * per_bit).sum()),
                          int(act.sum()), int(words.sum()), int((words.sum(1) * self.deg).sum()),
                          int(self.deg[act].sum()), int(scatter), 0)

    def _scatter(self):
        """pushes of the current frontier into self.next (gossip)"""
        vs, ms = np.nonzero(self.F)
        keys = set()
        for v, m in zip(vs, ms):
            d = self.deg[v]
            if d == 0:
                continue
            nb = self.g.colidx[self.g.rowptr[v]:self.g.rowptr[v + 1]]
            if d <= self.k:
                tg = nb
            else:
                pk = philox.gossip_picks(self.round, self.gid[v], m, d, self.k, self.gseed)[0]
                tg = nb[pk]
            for t in tg:
                if philox.churn_dropped(self.round, self.gid[v], self.gid[t], self.thr, self.cseed):
                    continue
                self.next[t, m] = True
                self.cand[t, m] = min(self.cand[t, m], self.gid[v])
                keys.add((v, t, m // 64))
        return len(keys)

    def step(self):
        V, M = self.V, self.M
        if self.round == 0:
            new = np.zeros((V, M), bool)
            new[self.src, np.arange(M)] = True
            self.seen |= new
            self.F = new
            self.hop[new] = 0
        elif self.mode == "flood":
            alive = ~philox.churn_dropped(self.round - 1, self.gid[self.rows], self.gid[self.g.colidx],
                                          self.thr, self.cseed)
            contrib = self.F[self.g.colidx] & alive[:, None]
            arr = np.zeros((V, M), bool)
            np.logical_or.at(arr, self.rows, contrib)
            new = arr & ~self.seen
            pend = new.copy()
            for e in range(len(self.rows)):  # ascending slots = ascending global ids per row
                u = self.rows[e]
                hit = contrib[e] & pend[u]
                if hit.any():
                    self.par[u, hit] = self.gid[self.g.colidx[e]]
                    pend[u] &= ~hit
            self.seen |= new
            self.hop[new] = self.round
            self.F = new
        else:
            new = self.next & ~self.seen
            self.par[new] = self.cand[new]
            self.cand[self.next] = np.iinfo(np.int64).max
            self.next[:] = False
            self.seen |= new
            self.hop[new] = self.round
            self.F = new
        per_bit = np.minimum(self.deg, self.k) if self.mode == "gossip" else np.maximum(self.deg - 1, 0)
        st = self._stats(new, per_bit)
        if self.mode == "gossip":
            st.scatter_words = self._scatter()
        self.round += 1
        return st

    def exchange_pack(self, plane, buf):
        if plane == 0:
            rows = self.F[self.send]
        else:
            rows = self.next[self.recv]
            self.next[self.recv] = False
        w = _words(rows).astype(np.int64).ravel()
        buf[:len(w)] = __import__("torch").from_numpy(w)

    def exchange_unpack(self, plane, buf):
        arr = buf.cpu().numpy().astype(np.int64).view(np.uint64)
        W = (self.M + 63) // 64
        if plane == 0:
            self.F[self.recv] = _bits(arr[:len(self.recv) * W].reshape(-1, W), self.M)
        else:
            b = _bits(arr[:len(self.send) * W].reshape(-1, W), self.M)
            # a boundary peer appears once per neighbouring rank: OR, never overwrite
            # (the device unpack uses atomicOr); gossip parents are not checked when partitioned
            np.logical_or.at(self.next, self.send, b)

    def exchange_pack_live(self, plane, buf):
        """The compacted records of include/p2pgpu.h p2pg_exchange_pack_live."""
        import torch
        W = (self.M + 63) // 64
        R = 1 + W
        if plane == 0:
            ids, off, rows = self.send, self.send_off, self.F[self.send]
        else:
            ids, off, rows = self.recv, self.recv_off, self.next[self.recv].copy()
            self.next[self.recv] = False
        words = _words(rows).astype(np.int64) if len(ids) else np.zeros((0, W), np.int64)
        counts = np.zeros(len(off) - 1, dtype=np.int64)
        out = buf.numpy() if not buf.is_cuda else None
        recs = np.zeros_like(out) if out is None else out
        for q in range(len(off) - 1):
            for i in range(off[q], off[q + 1]):
                if not rows[i].any():
                    continue
                r = (off[q] + counts[q]) * R
                recs[r] = i - off[q]
                recs[r + 1:r + R] = words[i]
                counts[q] += 1
        if out is None:
            buf.copy_(torch.from_numpy(recs))
        return counts

    def exchange_unpack_live(self, plane, buf, counts):
        arr = buf.cpu().numpy().astype(np.int64)
        W = (self.M + 63) // 64
        R = 1 + W
        ids, off = (self.recv, self.recv_off) if plane == 0 else (self.send, self.send_off)
        i = 0
        for p, n in enumerate(counts):
            for _ in range(int(n)):
                rec = arr[i * R:(i + 1) * R]
                v = ids[off[p] + rec[0]]
                b = _bits(rec[1:].view(np.uint64).reshape(1, W), self.M)[0]
                if plane == 0:
                    self.F[v] = b
                else:  # a boundary peer can be pushed to from several ranks: OR
                    self.next[v] |= b
                i += 1

    def deliveries(self, cap=None):
        """this round's first receipts (unordered contract: callers sort)"""
        from p2pnetwork.gpu.network import Deliveries
        vs, ms = np.nonzero(self.F)
        return Deliveries(vs.astype(np.int32), ms.astype(np.int32), self.hop[vs, ms].astype(np.int32),
                          self.par[vs, ms].astype(np.int32))

    def sends(self):
        """include/p2pgpu.h p2pg_get_sends: every send of the last round, sorted by (receiver,
        sender, msg); flood skips the connection a first receipt came from."""
        from p2pnetwork.gpu.network import Sends
        r = self.round - 1
        out = []
        for v, m in zip(*np.nonzero(self.F)):
            nb = self.g.colidx[self.g.rowptr[v]:self.g.rowptr[v + 1]]
            d = len(nb)
            if self.mode == "flood":
                tg = [u for u in nb if r == 0 or self.gid[u] != self.par[v, m]]
            elif d <= self.k:
                tg = list(nb)
            else:
                tg = list(nb[philox.gossip_picks(r, self.gid[v], m, d, self.k, self.gseed)[0]])
            for u in tg:
                lost = bool(philox.churn_dropped(r, self.gid[v], self.gid[u], self.thr, self.cseed))
                out.append((int(u), int(v), int(m), lost))
        out.sort()
        a = np.array(out, dtype=np.int64).reshape(-1, 4)
        return Sends(a[:, 1].astype(np.int32), a[:, 0].astype(np.int32), a[:, 2].astype(np.int32),
                     a[:, 3].astype(bool))

    def drop_relays(self, peer, msg):
        """p2pg_drop_relays: the listed first receipts of the last round do not relay."""
        peer, msg = np.asarray(peer, dtype=np.int64), np.asarray(msg, dtype=np.int64)
        assert self.F[peer, msg].all() and len(set(zip(peer.tolist(), msg.tolist()))) == len(peer)
        self.F[peer, msg] = False
        if self.mode == "gossip":  # redo the last round's pushes without them
            self.next[:] = False
            self.cand[:] = np.iinfo(np.int64).max
            self.round -= 1
            self._scatter()
            self.round += 1

    def update_edges(self, add=(), remove=()):
        """p2pg_update_edges between rounds: sends of the last round on removed connections
        are lost (flood: pulled over the new graph minus them next round; the mock keeps the
        plain form: static-topology tests only run through it mid-run)."""
        self.graph = self.g = self.g.with_changes(add, remove)
        self.deg = self.g.degree()
        self.rows = np.repeat(np.arange(self.V), self.deg)

    def seen_plane(self):
        return _words(self.seen)

    def hop_parent(self):
        return self.hop, self.par

    def close(self):
        pass
