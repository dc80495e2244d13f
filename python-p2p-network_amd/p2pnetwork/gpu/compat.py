"""Per-callback compatibility mode: ``Node``-subclass apps on a simulated peer graph.

``CompatNetwork`` builds one app object per peer of a ``PeerGraph`` and runs them round-
synchronously with the reference's hook semantics: every packet that arrives is counted
(``message_count_recv``) and handed to the receiver's ``node_message(connection, data)``
(NodeConnection.run, p2pnetwork/nodeconnection.py:211-216), duplicates included, and the app
alone decides what to send (README.md:20).  One Python call per arrival, so this is for small
graphs; the batched hook of ``GraphNetwork`` is the fast path.

Who carries the packets:

* The HIP engine carries every *relay it can express*: a broadcast originated with
  ``send_to_nodes(data)`` (node.py:106-112) becomes an engine message, and a first receipt of it
  that the app forwards the way the engine would -- flood: ``send_to_nodes(data, exclude=[the
  sender])``, or ``send_to_node`` on exactly those connections; gossip (build-defined, SURVEY.md
  A.3): ``send_to_nodes(data, ...)``, or ``send_to_node`` on exactly the k Philox picks -- stays
  in the engine's frontier.  A first receipt the app does not forward is withdrawn
  (``p2pg_drop_relays``).  The engine's sends of each round (``p2pg_get_sends``: every
  ``send_to_node`` call, the ones churn loses flagged) are the next round's arrivals.
* Every other send -- a different payload, a different target set, a second relay of the same
  message, a duplicate's relay, ``NodeConnection.send`` -- is carried by the host as an explicit
  packet, subject to the same churn rule.  For the dedup-relay apps of the reference's
  documentation and fixtures this path stays empty (``explicit_packets`` counts it).

Delivery order inside a round is the reference harness's: ascending receiver, then sender, then
the order the sender wrote the packets (its own hook order of the round before).  A connection's
byte stream is framed like NodeConnection.run, with its quirks: a body holding 0x04 arrives as
several packets, an empty packet (EOT at position 0) stops the stream for good
(nodeconnection.py:211).

What an app sees is the *contract* of the reference's hook surface:

* the hook names and the ``callback(event, main_node, connected_node, data)`` signature of
  node.py:25-29 (every hook fires the callback with the reference's argument shape);
* ``nodes_inbound`` / ``nodes_outbound`` / ``all_nodes`` (node.py:75-78), the message counters
  (node.py:65-67: send += 1 per ``send_to_node`` call before anything else, :116; recv += 1 per
  delivered packet, nodeconnection.py:215), ``send_to_nodes`` / ``send_to_node`` (node.py:106-120)
  and ``connect_with_node`` / ``disconnect_with_node`` (node.py:122-189);
* connection handles with ``id`` / ``host`` / ``port``, ``send``, ``set_info`` / ``get_info``.

Out of scope: sockets and threads, sha512 ids (a peer's id is its engine
index as a string), debug printing, pretty-printing.

Port an app by swapping its base class::

    from p2pnetwork.gpu.compat import SimNode as Node, CompatNetwork

    class MyNode(Node):
        def node_message(self, node, data):
            ...

    net = CompatNetwork(graph, MyNode)
    net.nodes[0].send_to_nodes({"mid": 1})    # queued; sent when run() starts (round 0)
    net.run()

Semantics beyond the hooks:

* Connections: for every edge {a, b} with a < b, a dialled b (a's ``nodes_outbound`` holds the
  handle to b, b's ``nodes_inbound`` the handle to a); both connected events fire per edge,
  ascending (a, b), at construction.
* ``run()`` sends what was queued since the previous ``run()`` in round 0 and runs rounds until
  nothing is in flight; rounds (``current_round``) and engine message ids count from 0 per run.
* Connection changes (also from inside ``node_message``) take effect between rounds through the
  engine's ``update_edges``: a removed connection loses the packets in flight on it and both ends
  see ``node_disconnected``; a new one fires the connected events when it appears.
"""
import threading

import numpy as np

from . import _lib, wire

# Lifecycle hooks and the shape of the callback they fire (node.py:282-352):
#   "conn"  -> callback(event, self, connection, {})
#   "error" -> callback(event, self, None, {"exception": exception})
#   "stop"  -> callback(event, self, {}, {})
_HOOK_SHAPES = {
    "outbound_node_connected": "conn",
    "inbound_node_connected": "conn",
    "inbound_node_disconnected": "conn",
    "outbound_node_disconnected": "conn",
    "node_disconnect_with_outbound_node": "conn",
    "outbound_node_connection_error": "error",
    "inbound_node_connection_error": "error",
    "node_request_to_stop": "stop",
}


def _lifecycle_hook(event, shape):
    if shape == "conn":
        def hook(self, node):
            self._emit(event, node, {})
    elif shape == "error":
        def hook(self, exception):
            self._emit(event, None, {"exception": exception})
    else:
        def hook(self):
            self._emit(event, {}, {})
    hook.__name__ = hook.__qualname__ = event
    hook.__doc__ = f"'{event}' event; override in a subclass, or receive it through callback."
    return hook


class SimConnection:
    """A peer's handle on one of its connections (what NodeConnection is to an app)."""

    def __init__(self, owner, peer, other):
        self.main_node = owner             # the node holding this handle
        self.peer = int(peer)              # engine index of the other end
        self.id, self.host, self.port = other.id, other.host, other.port
        self.info = {}
        self.terminate_flag = threading.Event()

    def send(self, data, encoding_type="utf-8", compression="none"):
        """NodeConnection.send (nodeconnection.py:107-160): one packet, no counter."""
        self.main_node._net._raw_send(self.main_node, self, data, encoding_type, compression)

    def parse_packet(self, packet):
        return wire.parse_packet(packet)

    def set_info(self, key, value):
        self.info[key] = value

    def get_info(self, key):
        return self.info[key]

    def stop(self):
        self.terminate_flag.set()

    def join(self, timeout=None):
        pass


class SimNode:
    """App base class for compat mode: the reference ``Node`` constructor signature, connection
    lists, counters, send calls and event hooks, with no server socket and no thread."""

    def __init__(self, host="127.0.0.1", port=0, id=None, callback=None, max_connections=0):
        self.host, self.port = host, port
        self.id = f"{host}:{port}" if id is None else str(id)
        self.callback = callback
        self.max_connections = max_connections
        self.nodes_inbound, self.nodes_outbound = [], []
        self.message_count_send = self.message_count_recv = self.message_count_rerr = 0
        self.terminate_flag = threading.Event()
        self._net, self._peer = None, -1  # bound by CompatNetwork

    @property
    def all_nodes(self):
        return self.nodes_inbound + self.nodes_outbound

    def _emit(self, event, node, data):
        if self.callback is not None:
            self.callback(event, self, node, data)

    # -- sends --------------------------------------------------------------------------------
    def send_to_nodes(self, data, exclude=[], compression="none"):
        self._net._broadcast_send(self, data, exclude, compression)

    def send_to_node(self, n, data, compression="none"):
        self._net._single_send(self, n, data, compression)

    # -- lifecycle: nothing to start or join ----------------------------------------------------
    def start(self):
        pass

    def join(self, timeout=None):
        pass

    def stop(self):
        self.node_request_to_stop()
        self.terminate_flag.set()

    def connect_with_node(self, host, port, reconnect=False):
        """Queue a connection to the simulated node at (host, port); it exists from the next
        round on.  Refused for ourselves; True if it already exists or is queued."""
        if (host, port) == (self.host, self.port):
            return False
        other = self._net._peer_at(host, port)
        if other is None:
            self.outbound_node_connection_error(ConnectionRefusedError(f"{host}:{port}"))
            return False
        if not self._net._is_linked(self._peer, other):
            self._net._queue_change(self._peer, other, True)
        return True

    def disconnect_with_node(self, node):
        """Close one of our outbound connections; it goes away between rounds (packets in
        flight on it are lost) and both ends then see node_disconnected."""
        if node not in self.nodes_outbound:
            return
        self.node_disconnect_with_outbound_node(node)
        node.stop()
        self._net._queue_change(self._peer, node.peer, False)

    def node_disconnected(self, node):
        for lst, hook in ((self.nodes_inbound, self.inbound_node_disconnected),
                          (self.nodes_outbound, self.outbound_node_disconnected)):
            if node in lst:
                lst.remove(node)
                hook(node)

    def node_message(self, node, data):
        self._emit("node_message", node, data)

    def node_reconnection_error(self, host, port, trials):
        return True


for _event, _shape in _HOOK_SHAPES.items():
    setattr(SimNode, _event, _lifecycle_hook(_event, _shape))
del _event, _shape


def _single_frame(pkt):
    """True if the receiver's framing yields exactly this one packet (no 0x04 inside the body,
    body not empty): only such payloads can be engine messages."""
    return len(pkt) > 1 and pkt.find(wire.EOT_CHAR) == len(pkt) - 1


class CompatNetwork:
    """A population of ``node_class`` instances over ``graph``, relayed by the HIP engine."""

    def __init__(self, graph, node_class=SimNode, mode="flood", fanout=3, host="127.0.0.1",
                 base_port=10000, node_kwargs=None, engine_factory=None, gossip_seed=0x5EED,
                 churn_threshold_value=0, churn_seed=0xC0FFEE, **engine_kw):
        from .network import GraphNetwork
        self.graph, self.mode, self.fanout = graph, mode, int(fanout)
        self.gossip_seed, self.churn_thr, self.churn_seed = int(gossip_seed), int(churn_threshold_value), int(churn_seed)
        kw = dict(node_kwargs or {})
        self.nodes = []
        for v in range(graph.V):
            n = node_class(host, base_port + v, str(v), **kw)
            n._net, n._peer = self, v
            self.nodes.append(n)
        self._by_addr = {(n.host, n.port): v for v, n in enumerate(self.nodes)}
        self._links = [dict() for _ in range(graph.V)]  # _links[v][u] = v's handle on u
        rp, ci = graph.rowptr, graph.colidx
        self._link_all((a, int(b)) for a in range(graph.V) for b in ci[rp[a]:rp[a + 1]] if b > a)
        self._deg = graph.degree()
        self._pending = {}   # {(min, max): (connect?, dialler, other)} for the next round boundary
        make = engine_factory or GraphNetwork
        engine_kw.setdefault("count_received", True)  # (small graphs: the churn count is cheap)
        self.engine = make(graph, mode=mode, fanout=fanout, gossip_seed=gossip_seed,
                           churn_threshold_value=churn_threshold_value, churn_seed=churn_seed,
                           **engine_kw)
        self.current_round = -1
        self.canonical_relays = 0   # first receipts relayed by the engine (its frontier)
        self.explicit_packets = 0   # packets the host carried (sends the engine cannot express)
        self._seq = 0
        self._q_orig = []           # queued originations: (peer, packet, seq)
        self._q_explicit = []       # queued explicit packets: (sender, receiver, seq, packet)
        self._streams = {}          # (sender, receiver) -> bytes not yet framed
        self._wedged = set()        # (sender, receiver) streams stopped by an empty packet
        self._ctx = None            # (receiver, sender, engine msg or None) during node_message
        self._first = {}            # engine first receipts of the round: (peer, msg) -> parent
        self._claims = {}           # (peer, msg) -> ("nodes", seq) | ("node", {target: seq})
        self._packets = []          # engine message -> its packet bytes
        self._engine_live = False   # the engine runs this run()'s broadcasts

    # -- wiring -------------------------------------------------------------------------------
    def _link_all(self, pairs):
        """Create both handles of each (dialler, listener) pair and fire the connected events."""
        for a, b in pairs:
            na, nb = self.nodes[a], self.nodes[b]
            ca, cb = SimConnection(na, b, nb), SimConnection(nb, a, na)
            na.nodes_outbound.append(ca)
            nb.nodes_inbound.append(cb)
            self._links[a][b], self._links[b][a] = ca, cb
            na.outbound_node_connected(ca)
            nb.inbound_node_connected(cb)

    def connection(self, a, b):
        """Peer a's handle on its connection to peer b (KeyError if there is none)."""
        return self._links[a][b]

    def _peer_at(self, host, port):
        return self._by_addr.get((host, port))

    def _is_linked(self, a, b):
        q = self._pending.get((min(a, b), max(a, b)))
        return q[0] if q is not None else b in self._links[a]

    def _queue_change(self, a, b, connect):
        """Latest request per pair wins; a request that restores the current state cancels.
        A connect remembers who asked: a is the dialler (outbound end, node.py:122-176)."""
        key = (min(a, b), max(a, b))
        if connect == (b in self._links[a]):
            self._pending.pop(key, None)
        else:
            self._pending[key] = (connect, a, b)

    def _apply_changes(self, in_flight=None):
        """Hand the queued changes to the engine (p2pg_update_edges), then mirror them on the
        node objects: removed handles + node_disconnected on both ends, new handles + the
        connected events (dialler outbound, other end inbound).  Packets in flight on a removed
        connection are lost (its reader stopped, nodeconnection.py:192-228)."""
        if not self._pending:
            return in_flight
        changes, self._pending = self._pending, {}
        add = [(a, b) for _, (c, a, b) in sorted(changes.items()) if c]  # (dialler, other)
        rem = sorted(k for k, (c, _, _) in changes.items() if not c)
        self.engine.update_edges(add=add, remove=rem)
        self.graph = self.engine.graph
        self._deg = self.graph.degree()
        gone = set()
        for a, b in rem:
            gone |= {(a, b), (b, a)}
            ca, cb = self._links[a].pop(b), self._links[b].pop(a)
            self.nodes[a].node_disconnected(ca)
            self.nodes[b].node_disconnected(cb)
            for k in ((a, b), (b, a)):
                self._streams.pop(k, None)
                self._wedged.discard(k)
        self._link_all(add)
        if in_flight is not None and gone:
            in_flight = [x for x in in_flight if (x[1], x[0]) not in gone]
        return in_flight

    # -- sends from app code --------------------------------------------------------------------
    def _next_seq(self):
        self._seq += 1
        return self._seq

    def _engine_msg_of(self, node, pkt):
        """The engine message this send may relay: the one being delivered to `node`, if the
        packet is that message's and `node` got it first this round (a first receipt)."""
        ctx = self._ctx
        if ctx is None or ctx[0] != node._peer or ctx[2] is None:
            return None
        m = ctx[2]
        if (node._peer, m) not in self._first or pkt != self._packets[m]:
            return None
        return m

    def _explicit(self, v, targets, seq, pkt):
        for u in targets:
            self._q_explicit.append((v, u, seq, pkt))
        self.explicit_packets += len(targets)

    def _broadcast_send(self, node, data, exclude, compression):
        """Node.send_to_nodes (node.py:106-112): send_to_node on every connection not excluded
        (identity filter), each counted before it is sent (:116)."""
        if node._net is not self:
            raise ValueError("node does not belong to this CompatNetwork")
        targets = [c for c in node.all_nodes if c not in exclude]
        pkt = wire.encode_packet(data, compression=compression)
        seq = self._next_seq()
        v = node._peer
        gossip = self.mode == "gossip"
        if self._ctx is None:
            if pkt is not None and not exclude and _single_frame(pkt):
                # a new broadcast: an engine message, originated in round 0 of the next run()
                node.message_count_send += min(self.fanout, len(targets)) if gossip else len(targets)
                self._q_orig.append((v, pkt, seq))
                return
            node.message_count_send += len(targets)
            if pkt is not None:
                self._explicit(v, [c.peer for c in targets], seq, pkt)
            return
        m = self._engine_msg_of(node, pkt) if pkt is not None else None
        if m is not None and (v, m) not in self._claims:
            deg = int(self._deg[v])
            if gossip:  # the gossip relay: the engine's k picks
                node.message_count_send += min(self.fanout, deg)
                self._claims[(v, m)] = ("nodes", seq)
                return
            parent = self._first[(v, m)]
            if len(targets) == deg - 1 and all(c.peer != parent for c in targets):
                node.message_count_send += len(targets)
                self._claims[(v, m)] = ("nodes", seq)
                return
        node.message_count_send += len(targets)
        if pkt is not None:
            self._explicit(v, [c.peer for c in targets], seq, pkt)

    def _single_send(self, node, conn, data, compression):
        """Node.send_to_node (node.py:114-120): counted first, sent only over a connection the
        node still has."""
        node.message_count_send += 1
        if conn not in node.all_nodes:
            return
        pkt = wire.encode_packet(data, compression=compression)
        seq = self._next_seq()
        if pkt is None:
            return
        v = node._peer
        m = self._engine_msg_of(node, pkt)
        if m is not None:
            c = self._claims.get((v, m))
            if c is None:
                c = self._claims[(v, m)] = ("node", {})
            if c[0] == "node" and conn.peer not in c[1]:
                c[1][conn.peer] = seq
                return
        self._explicit(v, [conn.peer], seq, pkt)

    def _raw_send(self, node, conn, data, encoding_type, compression):
        """NodeConnection.send called by the app itself: one packet, no counter."""
        pkt = wire.encode_packet(data, encoding_type, compression)
        seq = self._next_seq()
        if pkt is not None:
            self._explicit(node._peer, [conn.peer], seq, pkt)

    def gossip_connections(self, node, m):
        """The connections the engine's gossip picks for a first receipt of engine message m at
        `node` in the current round -- send_to_node on exactly these is relayed
        by the engine."""
        v = node._peer
        nb = self.graph.neighbours(v)
        out = np.zeros(max(self.fanout, 1), dtype=np.uint32)
        n = _lib.check(_lib.lib().p2pg_gossip_targets(max(self.current_round, 0), v, int(m), len(nb),
                                                      self.fanout, self.gossip_seed, _lib.ptr(out)))
        return [self._links[v][int(nb[j])] for j in out[:n]]

    # -- running --------------------------------------------------------------------------------
    def _lost(self, rnd, a, b):
        return self.churn_thr != 0 and _lib.lib().p2pg_churn_lost(rnd, a, b, self.churn_thr, self.churn_seed) != 0

    def _canonical(self, v, m, parent):
        """The targets of the engine's relay of first receipt (v, m)."""
        nb = self.graph.neighbours(v)
        if self.mode == "flood":
            return {int(u) for u in nb if u != parent}
        return {c.peer for c in self.gossip_connections(self.nodes[v], m)}

    def _resolve(self, rnd):
        """After a round's hooks: first receipts the app relayed as the engine would stay in its
        frontier (their sends get the seq of the app's call); the others are withdrawn, and their
        partial relays travel as explicit packets."""
        order, drop = {}, []
        for (v, m), parent in self._first.items():
            c = self._claims.get((v, m))
            if c is not None and c[0] == "nodes":
                order[(v, m)] = c[1]
                continue
            if c is not None and set(c[1]) == self._canonical(v, m, parent):
                order[(v, m)] = c[1]
                continue
            drop.append((v, m))
            if c is not None:
                for u, seq in c[1].items():
                    self._explicit(v, [u], seq, self._packets[m])
        self.canonical_relays += len(order)
        if drop:
            d = np.asarray(drop, dtype=np.int32).reshape(-1, 2)
            self.engine.drop_relays(d[:, 0], d[:, 1])
        return order

    def _in_flight(self, rnd, order):
        """The packets of round rnd: the engine's sends (after withdrawals) and the explicit
        ones, as (receiver, sender, seq, engine msg or None, packet, lost)."""
        out = []
        if order:
            s = self.engine.sends()
            for a, b, m, lost in zip(s.sender.tolist(), s.receiver.tolist(), s.msg.tolist(), s.lost.tolist()):
                o = order[(a, m)]
                out.append((b, a, o if isinstance(o, int) else o[b], m, self._packets[m], lost))
        for a, b, seq, pkt in self._q_explicit:
            out.append((b, a, seq, None, pkt, self._lost(rnd, a, b)))
        self._q_explicit = []
        return out

    def _deliver(self, arrivals):
        """NodeConnection.run for every connection, in the harness's order: bytes appended to
        the stream, framed on 0x04 (nodeconnection.py:204-214), each packet counted and handed to
        node_message (:215-216)."""
        for rcv, snd, _, m, pkt, lost in sorted(arrivals, key=lambda x: (x[0], x[1], x[2])):
            if lost:
                continue
            key = (snd, rcv)
            if key in self._wedged:
                continue
            conn = self._links[rcv].get(snd)
            if conn is None:
                continue
            buf = self._streams.pop(key, b"") + pkt
            packets, rest = wire.split_stream(buf)
            if rest:
                if rest[:1] == wire.EOT_CHAR:
                    self._wedged.add(key)  # eot_pos == 0: the loop never delivers again
                else:
                    self._streams[key] = rest
            node = self.nodes[rcv]
            one = len(packets) == 1 and not rest
            for p in packets:
                node.message_count_recv += 1
                self._ctx = (rcv, snd, m if one else None)
                try:
                    node.node_message(conn, wire.parse_packet(p))
                finally:
                    self._ctx = None

    def run(self, max_rounds=1 << 20):
        """Send what was queued since the last run (round 0), then deliver and dispatch round by
        round until nothing is in flight; returns the engine's per-round stats."""
        self._engine_live = False
        self._apply_changes()  # changes made before the run: its starting topology
        if not self._q_orig and not self._q_explicit:
            return []
        orig, self._q_orig = self._q_orig, []
        self._packets = [pkt for _, pkt, _ in orig]
        stats = []
        order = {}
        self.current_round = 0
        if orig:
            self.engine.broadcast(np.asarray([v for v, _, _ in orig], dtype=np.int32))
            self._engine_live = True
            st = self.engine.step()
            stats.append(st)
            order = {(v, m): seq for m, (v, _, seq) in enumerate(orig)}
            self.canonical_relays += len(orig)
        arrivals = self._in_flight(0, order)
        self.between_rounds(0)
        arrivals = self._apply_changes(arrivals)
        rnd = 0
        while any(not x[5] for x in arrivals) and rnd < max_rounds:
            rnd += 1
            self.current_round = rnd
            self._first, self._claims = {}, {}
            if self._engine_live and stats and stats[-1].active:
                st = self.engine.step()
                stats.append(st)
                if st.new_deliveries:
                    d = self.engine.deliveries()
                    self._first = dict(zip(zip(d.peer.tolist(), d.msg.tolist()), d.parent.tolist()))
            self._deliver(arrivals)
            order = self._resolve(rnd)
            arrivals = self._in_flight(rnd, order)
            self._first, self._claims = {}, {}
            self.between_rounds(rnd)
            arrivals = self._apply_changes(arrivals)
        return stats

    def between_rounds(self, rnd):
        """Called after round rnd's node_message calls, before queued connection changes are
        applied (override to drive topology changes from outside the nodes)."""

    def close(self):
        self.engine.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
