"""Per-callback compatibility mode: ``Node``-subclass apps on a simulated peer graph.

``CompatNetwork`` builds one app object per peer of a ``PeerGraph`` and drives them from the
HIP engine: every round's first receipts are handed to the receiving peer's
``node_message(connection, data)``, in a fixed order (ascending peer, then message), on the
calling thread.  One Python call per delivery, so this is for small graphs; the batched hook of
``GraphNetwork`` is the fast path.

What an app sees is the *contract* of the reference's hook surface, not
its implementation:

* the hook names and the ``callback(event, main_node, connected_node, data)`` signature of
  p2pnetwork/node.py:25-29 (every hook fires the callback with the reference's argument shape);
* ``nodes_inbound`` / ``nodes_outbound`` / ``all_nodes`` (node.py:75-78), the message counters
  (node.py:65-67), ``send_to_nodes`` / ``send_to_node`` (node.py:106-120) and
  ``connect_with_node`` / ``disconnect_with_node`` (node.py:122-189);
* connection handles with ``id`` / ``host`` / ``port``, ``send``, ``set_info`` / ``get_info``.

Out of scope: sockets and threads, sha512 ids (a peer's id is its engine
index as a string), debug printing, pretty-printing.

Port an app by swapping its base class::

    from p2pnetwork.gpu.compat import SimNode as Node, CompatNetwork

    class MyNode(Node):
        def node_message(self, node, data):
            ...

    net = CompatNetwork(graph, MyNode)
    net.nodes[0].send_to_nodes({"mid": 1})    # originates a broadcast
    net.run()

Semantics:

* Connections: for every edge {a, b} with a < b, a dialled b (a's ``nodes_outbound`` holds the
  handle to b, b's ``nodes_inbound`` the handle to a); both connected events fire per edge,
  ascending (a, b), at construction.
* Origination: ``send_to_nodes(data)`` outside a delivery queues a broadcast; ``run()`` relays
  the broadcasts queued since the previous ``run()`` (engine message ids count from 0 per run).
  Receivers get ``data`` after the wire codec (``wire.round_trip``: tuples arrive as lists, a str
  holding JSON arrives parsed); an unsendable payload reaches nobody (nodeconnection.py:158-160).
* Relay: the engine performs the dedup relay (flood: every connection but the sender; gossip:
  k Philox-chosen connections).  ``send_to_nodes`` / ``send_to_node`` made *inside*
  ``node_message`` are the app's relay of the message being delivered; they are absorbed
  (``CompatNetwork.absorbed_sends``), never sent twice.
* Counters: ``message_count_send`` = relays the engine made for the peer (every attempted send,
  also those churn drops, node.py:116); ``message_count_recv`` = its first receipts.
* Connection changes (also from inside ``node_message``) take effect between rounds through the
  engine's ``update_edges``: a removed connection loses the messages in flight on it and both
  ends see ``node_disconnected``; a new one fires the connected events when it appears.
"""
import threading

import numpy as np

from . import wire

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
        self.main_node._net._single_send(self.main_node, self, data, compression)

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
        """Close one of our outbound connections; it goes away between rounds (messages in
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


class CompatNetwork:
    """A population of ``node_class`` instances over ``graph``, relayed by the HIP engine."""

    def __init__(self, graph, node_class=SimNode, mode="flood", fanout=3, host="127.0.0.1",
                 base_port=10000, node_kwargs=None, engine_factory=None, **engine_kw):
        from .network import GraphNetwork
        self.graph, self.mode, self.fanout = graph, mode, int(fanout)
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
        self.engine = make(graph, mode=mode, fanout=fanout, **engine_kw)
        self.origins, self.payloads = [], []
        self._consumed = 0   # broadcasts relayed by earlier run() calls
        self.absorbed_sends = 0
        self.current_round = -1
        self._in_delivery = False

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

    def _apply_changes(self):
        """Hand the queued changes to the engine (p2pg_update_edges), then mirror them on the
        node objects: removed handles + node_disconnected on both ends, new handles + the
        connected events (dialler outbound, other end inbound)."""
        if not self._pending:
            return
        changes, self._pending = self._pending, {}
        add = [(a, b) for _, (c, a, b) in sorted(changes.items()) if c]  # (dialler, other)
        rem = sorted(k for k, (c, _, _) in changes.items() if not c)
        self.engine.update_edges(add=add, remove=rem)
        self.graph = self.engine.graph
        self._deg = self.graph.degree()
        for a, b in rem:
            ca, cb = self._links[a].pop(b), self._links[b].pop(a)
            self.nodes[a].node_disconnected(ca)
            self.nodes[b].node_disconnected(cb)
        self._link_all(add)

    # -- sends from app code --------------------------------------------------------------------
    def _broadcast_send(self, node, data, exclude, compression):
        if self._in_delivery:
            self.absorbed_sends += 1  # the engine already relays the message being delivered
            return
        if node._net is not self:
            raise ValueError("node does not belong to this CompatNetwork")
        if exclude:
            raise NotImplementedError("compat mode: a broadcast originates to every connection")
        ok, obj = wire.round_trip(data, compression=compression)
        if ok:
            self.origins.append(node._peer)
            self.payloads.append(obj)
        else:  # nothing reaches the wire, but every attempt is counted (node.py:116)
            node.message_count_send += len(node.all_nodes)

    def _single_send(self, node, conn, data, compression):
        if self._in_delivery:
            self.absorbed_sends += 1
            return
        raise NotImplementedError("compat mode: a single-connection send outside a delivery is not a "
                                  "broadcast; use send_to_nodes")

    # -- running --------------------------------------------------------------------------------
    def run(self, max_rounds=1 << 20):
        """Relay the broadcasts queued since the last run to quiescence, dispatching hooks per
        round; returns the engine's per-round stats."""
        self._apply_changes()  # changes made before the run: its starting topology
        base = self._consumed
        if base == len(self.origins):
            return []
        self._consumed = len(self.origins)
        self.engine.broadcast(np.asarray(self.origins[base:], dtype=np.int32))
        out = []
        while len(out) < max_rounds:
            st = self.engine.step()
            out.append(st)
            self.current_round = st.round
            if st.new_deliveries:
                d = self.engine.deliveries()
                for i in np.lexsort((d.msg, d.peer)):
                    self._deliver(int(d.peer[i]), base + int(d.msg[i]), int(d.parent[i]), st.round)
            self.between_rounds(st.round)
            self._apply_changes()  # made by this round's hooks: effective from the next round
            if not st.active:
                break
        return out

    def between_rounds(self, rnd):
        """Called after round rnd's node_message calls, before queued connection changes are
        applied (override to drive topology changes from outside the nodes)."""

    def _deliver(self, v, payload_idx, parent, rnd):
        node = self.nodes[v]
        deg = int(self._deg[v])
        if self.mode == "gossip":
            node.message_count_send += min(self.fanout, deg)
        else:
            node.message_count_send += deg if rnd == 0 else max(deg - 1, 0)
        if rnd == 0:
            return  # the origin's own send_to_nodes; it gets no node_message
        node.message_count_recv += 1
        self._in_delivery = True
        try:
            node.node_message(self._links[v][parent], self.payloads[payload_idx])
        finally:
            self._in_delivery = False

    def close(self):
        self.engine.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
