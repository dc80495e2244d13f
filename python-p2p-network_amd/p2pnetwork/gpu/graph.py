"""Peer graphs for the relay engine.

In p2pnetwork a peer's relay targets are ``Node.all_nodes`` = nodes_inbound + nodes_outbound
(p2pnetwork/node.py:75-78): every TCP connection relays in both directions, self connections
and duplicate connections are refused (node.py:131-139, :153).  A ``PeerGraph`` is that
topology for a whole population at once: an undirected simple graph in CSR form, neighbour
ids ascending (the lowest-id tie-break order), int64 row offsets and int32 peer ids.
"""
import ctypes

import numpy as np

from . import _lib


class PeerGraph:
    """Undirected simple peer graph in CSR form (rowptr int64 [V+1], colidx int32 [nnz])."""

    def __init__(self, rowptr, colidx, validate=True):
        self.rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        self.colidx = np.ascontiguousarray(colidx, dtype=np.int32)
        if validate:
            self.validate()

    @property
    def V(self):
        return len(self.rowptr) - 1

    @property
    def nnz(self):
        return int(self.rowptr[-1])

    @property
    def n_edges(self):
        return self.nnz // 2

    def degree(self):
        return np.diff(self.rowptr)

    def neighbours(self, v):
        return self.colidx[self.rowptr[v]:self.rowptr[v + 1]]

    def validate(self):
        rp, ci, V = self.rowptr, self.colidx, self.V
        if V < 1 or rp[0] != 0 or rp[-1] != len(ci) or np.any(np.diff(rp) < 0):
            raise ValueError("PeerGraph: malformed rowptr")
        if len(ci) and (ci.min() < 0 or ci.max() >= V):
            raise ValueError("PeerGraph: neighbour id out of range")
        rows = np.repeat(np.arange(V, dtype=np.int64), np.diff(rp))
        if np.any(rows == ci):
            raise ValueError("PeerGraph: self connection (refused by Node.connect_with_node)")
        same_row = rows[1:] == rows[:-1]
        if np.any(same_row & (ci[1:] <= ci[:-1])):
            raise ValueError("PeerGraph: rows must be strictly ascending (no duplicate connections)")
        # symmetric: every connection relays both ways (all_nodes = inbound + outbound)
        a = rows * V + ci
        b = ci.astype(np.int64) * V + rows
        if not np.array_equal(np.sort(a), np.sort(b)):
            raise ValueError("PeerGraph: adjacency must be symmetric")
        return self

    def with_changes(self, add=(), remove=()):
        """The topology after connecting the pairs in ``add`` and disconnecting those in
        ``remove`` (undirected (a, b) pairs) -- what GraphNetwork.update_edges applies."""
        V = self.V
        rows = np.repeat(np.arange(V, dtype=np.int64), self.degree())
        key = rows * V + self.colidx
        a = np.asarray(add, dtype=np.int64).reshape(-1, 2)
        r = np.asarray(remove, dtype=np.int64).reshape(-1, 2)
        rk = np.concatenate([r[:, 0] * V + r[:, 1], r[:, 1] * V + r[:, 0]])
        ak = np.concatenate([a[:, 0] * V + a[:, 1], a[:, 1] * V + a[:, 0]])
        key = np.union1d(np.setdiff1d(key, rk), ak)
        src, dst = key // V, key % V
        rowptr = np.zeros(V + 1, dtype=np.int64)
        np.cumsum(np.bincount(src, minlength=V), out=rowptr[1:])
        return PeerGraph(rowptr, dst.astype(np.int32))

    # ---- construction through the library's host generators ---------------------------
    @classmethod
    def _from_handle(cls, h):
        L = _lib.lib()
        V = ctypes.c_int64()
        nnz = ctypes.c_int64()
        _lib.check(L.p2pg_graph_info(h, ctypes.byref(V), ctypes.byref(nnz)))
        rp = ctypes.c_void_p()
        ci = ctypes.c_void_p()
        _lib.check(L.p2pg_graph_arrays(h, ctypes.byref(rp), ctypes.byref(ci)))
        rowptr = np.ctypeslib.as_array(ctypes.cast(rp, ctypes.POINTER(ctypes.c_int64)), (V.value + 1,)).copy()
        if nnz.value:
            colidx = np.ctypeslib.as_array(ctypes.cast(ci, ctypes.POINTER(ctypes.c_int32)), (nnz.value,)).copy()
        else:
            colidx = np.zeros(0, dtype=np.int32)
        L.p2pg_graph_free(h)
        return cls(rowptr, colidx, validate=False)

    @classmethod
    def generate(cls, kind, V, a=0.0, b=0.0, seed=1):
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.p2pg_graph_generate(int(kind), int(V), float(a), float(b), int(seed), ctypes.byref(h)))
        return cls._from_handle(h)

    @classmethod
    def random_regular(cls, V, d, seed=1):
        return cls.generate(_lib.GRAPH_RANDOM_REGULAR, V, d, 0.0, seed)

    @classmethod
    def gnp(cls, V, mean_degree, seed=1):
        """Erdos-Renyi G(n, p) with p = mean_degree / (V - 1)."""
        return cls.generate(_lib.GRAPH_GNP, V, mean_degree, 0.0, seed)

    @classmethod
    def barabasi_albert(cls, V, m, seed=1):
        return cls.generate(_lib.GRAPH_BARABASI_ALBERT, V, m, 0.0, seed)

    @classmethod
    def watts_strogatz(cls, V, k, beta, seed=1):
        return cls.generate(_lib.GRAPH_WATTS_STROGATZ, V, k, beta, seed)

    @classmethod
    def ring_chords(cls, V, stride=0):
        """Config 1 topology: ring plus chords (0, s), (s, 2s), ..."""
        return cls.generate(_lib.GRAPH_RING_CHORDS, V, stride, 0.0, 0)

    @classmethod
    def from_edges(cls, V, edges):
        e = np.asarray(edges, dtype=np.int32).reshape(-1, 2)
        a = np.ascontiguousarray(e[:, 0])
        b = np.ascontiguousarray(e[:, 1])
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().p2pg_graph_from_edges(int(V), len(a), _lib.ptr(a), _lib.ptr(b), ctypes.byref(h)))
        return cls._from_handle(h)


def make_sources(V, M, seed=1, msg_id_base=0):
    """Origin peer of each broadcast: lemire32(philox(key=(seed,'SRC'), ctr=(base+m,..)).x, V)."""
    out = np.zeros(M, dtype=np.int32)
    _lib.check(_lib.lib().p2pg_make_sources(int(V), int(M), int(seed), int(msg_id_base), _lib.ptr(out)))
    return out
