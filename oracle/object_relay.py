"""Object-level relay simulator (ORACLE -- test infrastructure / CPU baseline only).

Only tests/ and bench.py's cpu_baseline leg may import this module.  It is the 1-core, GIL-bound
analogue of what the reference does per relay (CPU baseline leg (i)):
one Python object per peer with an app-level ``seen`` dict (README.md:20), one object per
connection end, and per send the reference's work items --

  * Node.send_to_nodes -> Node.send_to_node per connection but the sender, counting
    message_count_send before sending                               (node.py:106-120)
  * NodeConnection.send: json.dumps(dict) + utf-8 + EOT 0x04 into the connection's stream
                                                                   (nodeconnection.py:128-143)
  * NodeConnection.run framing: split the stream on EOT, message_count_recv += 1,
    parse_packet = JSON-first decode, then node_message            (nodeconnection.py:167-218)

-- round-synchronous with receivers handling senders in ascending id, gossip /
churn as in SURVEY.md A.3 / A.4 (scalar pure-Python Philox).  Peers are instantiated when a
message first reaches them, so a bounded sample (``max_relays``) of a 10M-peer broadcast does
not build 10M objects.  Pinned against the reference-harness fixtures by
tests/test_object_relay.py.
"""
import json

EOT = b"\x04"
_MASK = 0xFFFFFFFF


def _philox(c0, c1, c2, c3, k0, k1):
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & _MASK, p1 & _MASK, ((p0 >> 32) ^ c3 ^ k1) & _MASK, p0 & _MASK
        k0 = (k0 + 0x9E3779B9) & _MASK
        k1 = (k1 + 0xBB67AE85) & _MASK
    return c0, c1, c2, c3


def _picks(rnd, peer, msg, n, k, seed):
    """Floyd + Lemire over Philox words; n > k."""
    out, words = [], None
    for i in range(k):
        if i % 4 == 0:
            words = _philox(rnd, peer, msg, 0x00475350 | ((i // 4) << 24), seed & _MASK, (seed >> 32) & _MASK)
        jmax = n - k + i
        t = (words[i % 4] * (jmax + 1)) >> 32
        out.append(jmax if t in out else t)
    return out


class _Conn:
    __slots__ = ("owner", "other", "sim")

    def __init__(self, owner, other, sim):
        self.owner, self.other, self.sim = owner, other, sim

    def send(self, data):  # NodeConnection.send for a dict payload
        self.sim.wire.setdefault((self.other, self.owner.id), bytearray()).extend(
            json.dumps(data).encode("utf-8") + EOT)


class _Peer:
    __slots__ = ("id", "nbrs", "conns", "seen", "count_send", "count_recv", "sim")

    def __init__(self, pid, nbrs, sim):
        self.id, self.nbrs, self.sim = pid, nbrs, sim
        self.conns = [_Conn(self, int(u), sim) for u in nbrs]  # all_nodes, ascending ids
        self.seen = {}
        self.count_send = self.count_recv = 0

    def node_message(self, conn, data):  # the dedup relay app
        mid = data["mid"]
        if mid in self.seen:
            return
        self.seen[mid] = (self.sim.round, conn.other)
        self.relay(data, conn)

    def relay(self, data, sender=None):
        sim = self.sim
        if sim.mode == "flood":
            for c in self.conns:  # send_to_nodes(data, exclude=[sender])
                if c is not sender:
                    self.send_to_node(c, data)
            return
        n = len(self.conns)
        chosen = self.conns if n <= sim.k else [self.conns[j] for j in
                                                 _picks(sim.round, self.id, data["mid"], n, sim.k, sim.gseed)]
        for c in chosen:
            self.send_to_node(c, data)

    def send_to_node(self, conn, data):
        self.count_send += 1  # counted before the send (node.py:116)
        sim = self.sim
        sim.sent += 1
        if sim.thr:
            a, b = (self.id, conn.other) if self.id < conn.other else (conn.other, self.id)
            if _philox(sim.round, a, b, 0x0043484E, sim.cseed & _MASK, (sim.cseed >> 32) & _MASK)[0] < sim.thr:
                return  # lost on a broken link
        conn.send(data)


class ObjectRelay:
    """Round-synchronous object-level relay over a CSR graph (rowptr, colidx)."""

    def __init__(self, rowptr, colidx, mode="flood", fanout=3, gossip_seed=0, churn_threshold=0,
                 churn_seed=0):
        self.rp, self.ci = rowptr, colidx
        self.mode, self.k, self.gseed = mode, int(fanout), int(gossip_seed)
        self.thr, self.cseed = int(churn_threshold), int(churn_seed)
        self.peers = {}
        self.wire = {}  # (receiver, sender) -> bytes sent this round
        self.round = 0
        self.sent = 0   # sum of message_count_send

    def peer(self, v):
        p = self.peers.get(v)
        if p is None:
            p = self.peers[v] = _Peer(v, self.ci[self.rp[v]:self.rp[v + 1]].tolist(), self)
        return p

    def run(self, src, max_relays=None):
        """Origins src[m] originate {"mid": m}; rounds until quiescence, or -- a bounded
        sample -- until max_relays sends have been made (mid-round).  Returns the relays of
        each round."""
        per_round = []
        self.round = 0
        for m, s in enumerate(src):
            p = self.peer(int(s))
            p.seen[m] = (0, -1)
            p.relay({"mid": m})
        per_round.append(self.sent)
        budget = max_relays if max_relays is not None else float("inf")
        while self.wire and self.sent < budget:
            self.round += 1
            batch, self.wire = self.wire, {}
            before = self.sent
            for (rcv, snd) in sorted(batch):  # receivers handle senders in ascending id
                if self.sent >= budget:
                    break
                node = self.peer(rcv)
                conn = node.conns[node.nbrs.index(snd)]
                buf = bytes(batch[(rcv, snd)])
                pos = buf.find(EOT)
                while pos > 0:  # NodeConnection.run framing
                    packet, buf = buf[:pos], buf[pos + 1:]
                    node.count_recv += 1
                    node.node_message(conn, json.loads(packet.decode("utf-8")))
                    pos = buf.find(EOT)
            per_round.append(self.sent - before)
        return per_round

    def planes(self, V, M):
        """hop / parent [V][M] (numpy int32, -1 = not delivered / origin)."""
        import numpy as np
        hop = np.full((V, M), -1, dtype=np.int32)
        par = np.full((V, M), -1, dtype=np.int32)
        for v, p in self.peers.items():
            for m, (r, s) in p.seen.items():
                hop[v, m], par[v, m] = r, s
        return hop, par
