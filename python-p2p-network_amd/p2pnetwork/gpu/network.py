"""GraphNetwork: a whole population of relaying p2pnetwork peers on one MI355X.

What an application builds on p2pnetwork for a broadcast is (pj8912/python-p2p-network):

    class MyNode(Node):                                   # p2pnetwork/node.py:13
        def node_message(self, node, data):               # node.py:334-338
            if data["id"] in self.seen: return            # dedup, README.md:20
            self.seen.add(data["id"])
            self.send_to_nodes(data, exclude=[node])      # node.py:106-112 -> send_to_node
                                                          #   (message_count_send += 1, :116)

GraphNetwork runs that relay for every peer of a ``PeerGraph`` at once, for up to thousands of
concurrent broadcasts (64 per uint64 word), round-synchronously, through the HIP engine behind
the C-ABI of include/p2pgpu.h.  The hook surface is kept in batched form: per round,
``node_message_batch(deliveries)`` receives the first receipts of that round as arrays
(peer, msg, hop, parent) -- the node_message events that pass dedup -- and a
``callback(event, network, connected_node, data)`` with the reference signature
(node.py:25-29) is invoked with event "node_message_batch".  Per-callback replay for Node
subclasses is in ``p2pnetwork.gpu.compat``.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .graph import PeerGraph

# p2pg_round_stats.push_form (include/p2pgpu.h P2PG_PUSH_*)
PUSH_FORMS = ("none", "atomic", "edge", "fused", "update_edge")

STAT_FIELDS = ("round", "active", "new_deliveries", "relays", "active_vertices", "active_words",
               "wedges", "deg_active", "scatter_words", "touched_words", "received")


@dataclass(slots=True)
class RoundStats:
    round: int
    active: int
    new_deliveries: int
    relays: int
    active_vertices: int
    active_words: int
    wedges: int
    deg_active: int
    scatter_words: int
    touched_words: int
    received: int = 0   # packets that arrived this round (sum of message_count_recv += 1,
                        # nodeconnection.py:215): last round's sends less the lost ones
    push_form: int = 0  # gossip: how this round's pushes left (PUSH_FORMS); not a result
    received_exact: int = 1  # 0: a churn run without count_received -- `received` is then the
                             # sends of the round before (an upper bound)

    @classmethod
    def from_c(cls, s):
        return cls(*(int(getattr(s, f)) for f in STAT_FIELDS), push_form=int(s.push_form),
                   received_exact=int(s.received_exact))

    @classmethod
    def from_c_array(cls, buf, n):
        """The first n entries of a RoundStatsC array (one numpy view instead of 11 ctypes field
        reads per round: p2pg_run's results are converted while the GPU waits for the next call)."""
        if n <= 0:
            return []
        rows = np.frombuffer(buf, dtype=_ROUND_DTYPE, count=n)[_ROUND_COLS].tolist()
        return [cls(*r) for r in rows]

    def as_dict(self):
        return {f: getattr(self, f) for f in STAT_FIELDS}


@dataclass
class Sends:
    """Every send of one round (Node.send_to_node calls, node.py:114-120), sorted by (receiver,
    sender, msg); lost = churn dropped it (nodeconnection.py:123-126).  The ones not lost are the
    next round's arrivals, each a node_message call (nodeconnection.py:211-216)."""
    sender: np.ndarray
    receiver: np.ndarray
    msg: np.ndarray
    lost: np.ndarray

    def __len__(self):
        return len(self.sender)


@dataclass
class Deliveries:
    """First receipts of one round, sorted by (peer, msg); parent = -1 at the origin."""
    peer: np.ndarray
    msg: np.ndarray
    hop: np.ndarray
    parent: np.ndarray

    def __len__(self):
        return len(self.peer)


# index of SnapHeader.total_relays in the snapshot header viewed as uint64 words (engine.cpp:
# magic 0, version/mode 1, V 2, nnz 3, M/W 4, fanout/round 5, flags/thr 6, base/done 7,
# consume/has_next 8, gossip_seed 9, churn_seed 10, graph_hash 11, src_hash 12, total_relays 13)
_SNAP_TOTAL_RELAYS_WORD = 13


def churn_threshold(p_drop):
    """floor(p_drop * 2^32), the integer threshold of the per-round edge-drop mask."""
    if not 0.0 <= p_drop < 1.0:
        raise ValueError("churn probability must be in [0, 1)")
    return int(np.floor(p_drop * 4294967296.0))


_ROUND_DTYPE = np.dtype([(n, {ctypes.c_int32: "<i4", ctypes.c_uint64: "<u8"}[t])
                         for n, t in _lib.RoundStatsC._fields_])
assert _ROUND_DTYPE.itemsize == ctypes.sizeof(_lib.RoundStatsC)
_ROUND_COLS = list(STAT_FIELDS) + ["push_form", "received_exact"]


class GraphNetwork:
    """A peer graph resident in HBM plus the relay engine that floods/gossips over it."""

    def __init__(self, graph, mode="flood", fanout=3, gossip_seed=0x5EED, churn=0.0,
                 churn_threshold_value=None, churn_seed=0xC0FFEE, record=False, timing=False,
                 device=0, msg_id_base=0, callback=None, autostop=True, local_graph=False,
                 count_received=False):
        if not isinstance(graph, PeerGraph):
            raise TypeError("graph must be a PeerGraph")
        if mode not in ("flood", "gossip"):
            raise ValueError("mode must be 'flood' or 'gossip'")
        self.graph = graph
        self.mode = mode
        self.fanout = int(fanout)
        self.record = bool(record)
        self.callback = callback
        cfg = _lib.Config()
        cfg.mode = _lib.MODE_FLOOD if mode == "flood" else _lib.MODE_GOSSIP
        cfg.fanout = self.fanout
        cfg.gossip_seed = int(gossip_seed)
        cfg.churn_seed = int(churn_seed)
        cfg.churn_threshold = int(churn_threshold_value if churn_threshold_value is not None
                                  else churn_threshold(churn))
        cfg.msg_id_base = int(msg_id_base)
        cfg.flags = ((_lib.FLAG_RECORD if record else 0) | (_lib.FLAG_TIMING if timing else 0)
                     | (0 if autostop else _lib.FLAG_NO_AUTOSTOP)
                     | (_lib.FLAG_LOCAL_GRAPH if local_graph else 0)
                     | (_lib.FLAG_RECEIVED if count_received else 0))
        cfg.device = int(device)
        self.config = cfg
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.p2pg_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self._check(L.p2pg_load_csr(h, graph.V, _lib.ptr(graph.rowptr), _lib.ptr(graph.colidx)))
        self.sources = None
        self.rounds = []
        self.message_count_send = 0  # sum of Node.message_count_send (node.py:65, :116)
        self._run_buf = None

    # -- plumbing -------------------------------------------------------------------------
    def _check(self, rc):
        return _lib.check(rc, self._h)

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().p2pg_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def M(self):
        return 0 if self.sources is None else len(self.sources)

    @property
    def W(self):
        return (self.M + 63) // 64

    def set_stream(self, hip_stream):
        """Launch on an external hipStream_t handle (int), e.g. torch's current stream."""
        self._check(_lib.lib().p2pg_set_stream(self._h, ctypes.c_void_p(hip_stream or None)))

    # -- broadcasts -----------------------------------------------------------------------
    def broadcast(self, sources):
        """Originate one broadcast per entry (origin peer ids); message m = position m.
        Equivalent of calling Node.send_to_nodes(data) at each origin (node.py:106)."""
        src = np.ascontiguousarray(sources, dtype=np.int32)
        if src.ndim != 1 or len(src) == 0:
            raise ValueError("sources must be a non-empty 1-D array of peer ids")
        self._check(_lib.lib().p2pg_set_sources(self._h, len(src), _lib.ptr(src)))
        self.sources = src
        self.rounds = []
        self.message_count_send = 0

    def reset(self):
        self._check(_lib.lib().p2pg_reset(self._h))
        self.rounds = []
        self.message_count_send = 0

    def step_begin(self):
        """Start the next round asynchronously: on a vertex-partitioned rank, the peers with no
        ghost neighbour (p2pg_step_begin); ``step`` / ``step_end`` finishes the round."""
        self._check(_lib.lib().p2pg_step_begin(self._h))

    def step_end(self):
        return self.step()

    def step(self):
        """Run one round; returns its RoundStats (``active`` = messages still in flight)."""
        s = _lib.RoundStatsC()
        self._check(_lib.lib().p2pg_step(self._h, ctypes.byref(s)))
        st = RoundStats.from_c(s)
        self.rounds.append(st)
        self.message_count_send += st.relays
        if st.new_deliveries and self._wants_deliveries():
            self.node_message_batch(self.deliveries())
        return st

    def run(self, max_rounds=1 << 20):
        """Rounds until quiescence; returns the list of RoundStats (last one has no receipts)."""
        if not self._wants_deliveries():
            buf = self._run_buf
            if buf is None:  # (kept: a fresh 4096-entry array per call costs ~20 us of host time)
                buf = self._run_buf = (_lib.RoundStatsC * 4096)()
            out = []
            while len(out) < max_rounds:
                n = ctypes.c_int32()
                chunk = min(max_rounds - len(out), len(buf))
                rc = _lib.lib().p2pg_run(self._h, chunk, buf, ctypes.byref(n))
                got = RoundStats.from_c_array(buf, n.value)  # rounds that stand are kept even
                out.extend(got)                              # if the call failed
                self.rounds.extend(got)
                self.message_count_send += sum(st.relays for st in got)
                rc = self._check(rc)
                if rc == 0 or n.value == 0:
                    break
            return out
        out = []
        while len(out) < max_rounds:
            st = self.step()
            out.append(st)
            if not st.active:
                break
        return out

    # -- topology changes between rounds ------------------------------
    def update_edges(self, add=(), remove=()):
        """Connect the (a, b) pairs in ``add`` (Node.connect_with_node, node.py:122-176) and
        disconnect those in ``remove`` (Node.disconnect_with_node, node.py:178-189) between
        rounds.  Messages in flight on a removed connection are lost; every send from the next
        round on uses the new connections (include/p2pgpu.h p2pg_update_edges)."""
        a = np.ascontiguousarray(np.asarray(add, dtype=np.int32).reshape(-1, 2))
        r = np.ascontiguousarray(np.asarray(remove, dtype=np.int32).reshape(-1, 2))
        self._check(_lib.lib().p2pg_update_edges(self._h, len(a), _lib.ptr(a) if len(a) else None,
                                                 len(r), _lib.ptr(r) if len(r) else None))
        self.graph = self.graph.with_changes(a, r)

    def connect(self, pairs):
        self.update_edges(add=pairs)

    def disconnect(self, pairs):
        self.update_edges(remove=pairs)

    # -- snapshot / resume ------------------------------------------
    def snapshot(self):
        """The run state between rounds as a uint8 array (p2pg_snapshot)."""
        n = ctypes.c_int64()
        self._check(_lib.lib().p2pg_snapshot_size(self._h, ctypes.byref(n)))
        buf = np.empty(max(n.value, 1), dtype=np.uint8)
        self._check(_lib.lib().p2pg_snapshot(self._h, _lib.ptr(buf), n.value))
        return buf[:n.value]

    def restore(self, buf):
        """Continue from a snapshot of an engine with the same configuration, graph and
        sources (call broadcast(sources) first)."""
        b = np.ascontiguousarray(buf, dtype=np.uint8)
        self._check(_lib.lib().p2pg_restore(self._h, _lib.ptr(b), len(b)))
        self.rounds = []
        self.message_count_send = int(np.frombuffer(b[:128].tobytes(), dtype=np.uint64)[
            _SNAP_TOTAL_RELAYS_WORD])

    def save_snapshot(self, path):
        np.save(path, self.snapshot(), allow_pickle=False)

    def load_snapshot(self, path):
        self.restore(np.load(path, allow_pickle=False))

    # -- the batched hook (override like Node.node_message, node.py:334-338) --------------
    def node_message_batch(self, deliveries):
        if self.callback is not None:
            self.callback("node_message_batch", self, None, deliveries)

    def _wants_deliveries(self):
        return (self.callback is not None
                or type(self).node_message_batch is not GraphNetwork.node_message_batch)

    def deliveries_count(self):
        """Number of first-receipt records the last round's delivery stream holds."""
        n = ctypes.c_int64()
        z = np.zeros(1, dtype=np.int32)
        self._check(_lib.lib().p2pg_get_new_deliveries(self._h, 0, _lib.ptr(z), _lib.ptr(z), _lib.ptr(z),
                                                        _lib.ptr(z), ctypes.byref(n)))
        return int(n.value)

    def deliveries(self, cap=None):
        """First receipts of the most recent round as (peer, msg, hop, parent) arrays."""
        if cap is None:
            cap = self.rounds[-1].new_deliveries if self.rounds else 0
        cap = int(cap)
        peer = np.zeros(max(cap, 1), dtype=np.int32)
        msg = np.zeros_like(peer)
        hop = np.zeros_like(peer)
        parent = np.zeros_like(peer)
        n = ctypes.c_int64()
        self._check(_lib.lib().p2pg_get_new_deliveries(
            self._h, cap, _lib.ptr(peer), _lib.ptr(msg), _lib.ptr(hop), _lib.ptr(parent), ctypes.byref(n)))
        k = min(n.value, cap)
        return Deliveries(peer[:k], msg[:k], hop[:k], parent[:k])

    def sends(self):
        """Every send of the most recent round (p2pg_get_sends): the packets its first receipts
        put on the wire, duplicates included, after any drop_relays."""
        n = ctypes.c_int64()
        z = np.zeros(1, dtype=np.int32)
        z8 = np.zeros(1, dtype=np.uint8)
        L = _lib.lib()
        self._check(L.p2pg_get_sends(self._h, 0, _lib.ptr(z), _lib.ptr(z), _lib.ptr(z), _lib.ptr(z8),
                                     ctypes.byref(n)))
        cap = int(n.value)
        snd = np.zeros(max(cap, 1), dtype=np.int32)
        rcv = np.zeros_like(snd)
        msg = np.zeros_like(snd)
        lost = np.zeros(max(cap, 1), dtype=np.uint8)
        self._check(L.p2pg_get_sends(self._h, cap, _lib.ptr(snd), _lib.ptr(rcv), _lib.ptr(msg), _lib.ptr(lost),
                                     ctypes.byref(n)))
        k = min(int(n.value), cap)
        return Sends(snd[:k], rcv[:k], msg[:k], lost[:k].astype(bool))

    def drop_relays(self, peer, msg):
        """Withdraw the relays of these first receipts of the most recent round: the app did not
        forward them (p2pg_drop_relays)."""
        p = np.ascontiguousarray(peer, dtype=np.int32)
        m = np.ascontiguousarray(msg, dtype=np.int32)
        if len(p) != len(m):
            raise ValueError("peer and msg must have the same length")
        self._check(_lib.lib().p2pg_drop_relays(self._h, len(p), _lib.ptr(p) if len(p) else None,
                                                _lib.ptr(m) if len(m) else None))
        drop = sum(min(self.fanout, d) if self.mode == "gossip" else
                   (d if self.rounds and self.rounds[-1].round == 0 else max(d - 1, 0))
                   for d in self.graph.degree()[p].tolist())
        self.message_count_send -= drop

    # -- validation planes ----------------------------------------------------------------
    def seen_plane(self):
        out = np.zeros((self.graph.V, self.W), dtype=np.uint64)
        self._check(_lib.lib().p2pg_read_planes(self._h, _lib.ptr(out), None, None))
        return out

    def seen_word(self, w):
        """uint64 [V]: word w of every peer's seen row (messages 64w .. 64w+63), without
        copying the whole plane (p2pg_read_seen_word)."""
        out = np.zeros(self.graph.V, dtype=np.uint64)
        self._check(_lib.lib().p2pg_read_seen_word(self._h, int(w), _lib.ptr(out)))
        return out

    def delivered(self):
        """bool [V, M]: peer v has received broadcast m (its dedup 'seen' set)."""
        s = self.seen_plane()
        bits = np.unpackbits(s.view(np.uint8).reshape(self.graph.V, -1), axis=1, bitorder="little")
        return bits[:, :self.M].astype(bool)

    def hop_parent(self):
        """(hop, parent) int32 [V, M]; needs record=True.  -1 = not delivered / origin."""
        if not self.record:
            raise RuntimeError("hop/parent planes need GraphNetwork(record=True)")
        hop = np.zeros((self.graph.V, self.M), dtype=np.int32)
        par = np.zeros_like(hop)
        self._check(_lib.lib().p2pg_read_planes(self._h, None, _lib.ptr(hop), _lib.ptr(par)))
        return hop, par

    KERNEL_CLASSES = ("seed", "flood_pull", "gossip_scatter_atomic", "record", "gossip_update",
                      "gossip_pull", "gossip_scatter_store", "gossip_fused")

    def kernel_times(self):
        """Summed device ms and launch counts per kernel class since the last reset (needs
        timing=True); classes as in include/p2pgpu.h (P2PG_KCLASS_N)."""
        n = len(self.KERNEL_CLASSES)
        ms = np.zeros(n, dtype=np.float64)
        cnt = np.zeros(n, dtype=np.int64)
        self._check(_lib.lib().p2pg_kernel_times(self._h, _lib.ptr(ms), _lib.ptr(cnt)))
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(self.KERNEL_CLASSES)}

    def set_timed_classes(self, classes=None):
        """Time only these kernel classes with HIP events (None = all; p2pg_set_timed_classes):
        events cost stream time, so a measurement can bracket its dominant kernel alone."""
        names = self.KERNEL_CLASSES if classes is None else classes
        mask = 0
        for k in names:
            mask |= 1 << self.KERNEL_CLASSES.index(k)
        self._check(_lib.lib().p2pg_set_timed_classes(self._h, mask))

    # -- vertex-partitioned runs (p2pnetwork.gpu.partition) --------------------------------
    def set_global_ids(self, gid):
        self._gid = np.ascontiguousarray(gid, dtype=np.int32)
        self._check(_lib.lib().p2pg_set_global_ids(self._h, _lib.ptr(self._gid)))

    def set_ghost_senders(self, ghost_deg, slot_pos):
        """Partitioned gossip records / deliveries: the ghosts' global degrees and, per local
        slot, the row owner's position in its ghost neighbour's global adjacency (-1 = local
        neighbour) -- p2pg_set_ghost_senders."""
        self._gdeg = np.ascontiguousarray(ghost_deg, dtype=np.int32)
        self._gpos = np.ascontiguousarray(slot_pos, dtype=np.int32)
        self._check(_lib.lib().p2pg_set_ghost_senders(self._h, _lib.ptr(self._gdeg), _lib.ptr(self._gpos)))

    def set_exchange(self, send_local, recv_local):
        s = np.ascontiguousarray(send_local, dtype=np.int32)
        r = np.ascontiguousarray(recv_local, dtype=np.int32)
        self._check(_lib.lib().p2pg_set_exchange(self._h, len(s), _lib.ptr(s), len(r), _lib.ptr(r)))

    def set_exchange_segments(self, send_counts, recv_counts):
        """Rows per rank of the send / recv lists (p2pg_set_exchange_segments)."""
        sc = np.ascontiguousarray(send_counts, dtype=np.int64)
        rc = np.ascontiguousarray(recv_counts, dtype=np.int64)
        self._nseg = len(sc)
        self._check(_lib.lib().p2pg_set_exchange_segments(self._h, len(sc), _lib.ptr(sc), _lib.ptr(rc)))

    def exchange_pack_live(self, plane, buf):
        """Pack the live rows of the last round as records into device buffer ``buf``; returns
        the record count per destination rank (p2pg_exchange_pack_live)."""
        counts = np.zeros(self._nseg, dtype=np.int64)
        self._check(_lib.lib().p2pg_exchange_pack_live(self._h, int(plane), ctypes.c_void_p(buf.data_ptr()),
                                                       _lib.ptr(counts)))
        return counts

    def set_exchange_buffer(self, plane, buf):
        """Pack the live rows of ``plane`` into device buffer ``buf`` inside every round, their
        counts read back with the round counters (p2pg_set_exchange_buffer); ``None`` = off."""
        self._check(_lib.lib().p2pg_set_exchange_buffer(
            self._h, int(plane), ctypes.c_void_p(buf.data_ptr()) if buf is not None else None))

    def exchange_unpack_live(self, plane, buf, counts):
        c = np.ascontiguousarray(counts, dtype=np.int64)
        self._check(_lib.lib().p2pg_exchange_unpack_live(self._h, int(plane), ctypes.c_void_p(buf.data_ptr()),
                                                         _lib.ptr(c)))

    def alloc_exchange(self, n_words):
        """Device buffer for exchange rows (a torch tensor on this engine's GPU)."""
        import torch
        return torch.empty(max(int(n_words), 1), dtype=torch.int64, device=f"cuda:{self.config.device}")

    def exchange_pack(self, plane, buf):
        self._check(_lib.lib().p2pg_exchange_pack(self._h, int(plane), ctypes.c_void_p(buf.data_ptr())))

    def exchange_unpack(self, plane, buf):
        self._check(_lib.lib().p2pg_exchange_unpack(self._h, int(plane), ctypes.c_void_p(buf.data_ptr())))

    def device_philox(self, ctr, key):
        """Evaluate Philox4x32-10 on the GPU for counters [n, 4] (KAT hook)."""
        c = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
        k = np.ascontiguousarray(key, dtype=np.uint32)
        out = np.zeros_like(c)
        self._check(_lib.lib().p2pg_device_philox(self._h, len(c), _lib.ptr(c), _lib.ptr(k), _lib.ptr(out)))
        return out
