"""Per-callback compatibility mode: existing ``Node``-subclass apps on a simulated graph.

``SimNode`` has the hook surface of ``p2pnetwork.node.Node`` (node.py:13-363) without sockets
or threads; ``CompatNetwork`` builds one per peer of a ``PeerGraph``, wires ``SimConnection``
stand-ins for ``NodeConnection`` (nodeconnection.py:8-50) and drives them from the HIP engine:
each round's first receipts become ``node_message(connection, data)`` calls on the receiving
node, in a deterministic order (ascending peer, then message), on the calling thread.  Meant
for small graphs (one Python call per delivery); the batched hook of ``GraphNetwork`` is the
fast path.

An app ports by swapping its base class::

    from p2pnetwork.gpu.compat import SimNode as Node, CompatNetwork

    class MyNode(Node):                       # unchanged app code (README.md:35-76)
        def node_message(self, node, data):
            ...

    net = CompatNetwork(graph, MyNode)
    net.nodes[0].send_to_nodes({"mid": 1})    # originates a broadcast (node.py:106-112)
    net.run()

Semantics (compat mode):

* Connections: for every edge {a, b} with a < b, a dialled b -- ``a.nodes_outbound`` holds the
  connection to b, ``b.nodes_inbound`` the one to a -- and ``outbound_node_connected`` /
  ``inbound_node_connected`` fire once per connection, ascending (a, b), at construction.
* Origination: ``send_to_nodes(data)`` on a node outside a delivery originates a broadcast
  (the engine's message id = call order).  The payload every receiver sees is ``data`` after
  the wire codec (``wire.round_trip``: what ``NodeConnection.send`` + ``parse_packet``
  produce, so tuples arrive as lists, a str holding JSON arrives parsed, ...); an unsendable
  payload reaches nobody, as in the reference (nodeconnection.py:158-160).
* Relay: the engine performs the dedup relay (flood: all connections but the sender; gossip:
  k Philox-chosen connections).  ``send_to_nodes`` / ``send_to_node`` called *inside*
  ``node_message`` are the app's relay of the message being delivered and are absorbed
  (counted in ``CompatNetwork.absorbed_sends``), never sent twice; the payload cannot be
  changed per hop.
* Counters: ``message_count_send`` = the relays the engine made for the node (node.py:116
  semantics: every attempted send, also those churn drops); ``message_count_recv`` = its
  deliveries (first receipts -- duplicates are dropped by the engine before any hook).
* Lifecycle: ``start`` / ``join`` are no-ops; ``stop`` fires ``node_request_to_stop``.
* Connection changes: ``connect_with_node(host, port)`` / ``disconnect_with_node(conn)`` (also
  from inside ``node_message``) take effect between rounds through the engine's
  ``update_edges``: connected events fire then; a removed connection loses the messages in
  flight on it and both ends get ``node_disconnected`` (node.py:122-189, :307-319).
"""
import hashlib
import random
import threading

import numpy as np

from . import wire


class SimConnection:
    """One end of a connection, as seen from ``main_node`` (the NodeConnection stand-in)."""

    def __init__(self, main_node, peer, id, host, port):
        self.main_node = main_node
        self.peer = int(peer)          # engine peer id of the other end
        self.id = str(id)              # nodeconnection.py:37 (the other node's id)
        self.host, self.port = host, port
        self.info = {}                 # nodeconnection.py:42
        self.terminate_flag = threading.Event()
        self.EOT_CHAR, self.COMPR_CHAR = wire.EOT_CHAR, wire.COMPR_CHAR

    def send(self, data, encoding_type="utf-8", compression="none"):
        self.main_node._net._conn_send(self.main_node, self, data, compression)

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

    def __str__(self):
        return f"NodeConnection: {self.main_node.host}:{self.main_node.port} <-> {self.host}:{self.port} ({self.id})"

    def __repr__(self):
        return f"<NodeConnection: Node {self.main_node.host}:{self.main_node.port} <-> Connection {self.host}:{self.port}>"


class SimNode:
    """``Node``'s app-facing surface (node.py:13-363) for compat mode: same constructor
    signature, attributes, send methods and event hooks; no server socket, no thread."""

    def __init__(self, host="127.0.0.1", port=0, id=None, callback=None, max_connections=0):
        self.terminate_flag = threading.Event()
        self.host, self.port = host, port
        self.callback = callback
        self.nodes_inbound = []
        self.nodes_outbound = []
        self.reconnect_to_nodes = []
        self.id = self.generate_id() if id is None else str(id)
        self.message_count_send = 0
        self.message_count_recv = 0
        self.message_count_rerr = 0
        self.max_connections = max_connections
        self.debug = False
        self._net = None  # set by CompatNetwork

    @property
    def all_nodes(self):
        return self.nodes_inbound + self.nodes_outbound

    def debug_print(self, message):
        if self.debug:
            print(f"DEBUG ({self.id}): {message}")

    def generate_id(self):
        h = hashlib.sha512()
        h.update((self.host + str(self.port) + str(random.randint(1, 99999999))).encode("ascii"))
        return h.hexdigest()

    def print_connections(self):
        print("Node connection overview:")
        print(f"Total nodes connected with us: {len(self.nodes_inbound)}")
        print(f"Total nodes connected to     : {len(self.nodes_outbound)}")

    # -- sending (node.py:106-120) ----------------------------------------------------------
    def send_to_nodes(self, data, exclude=[], compression="none"):
        self._net._send_to_nodes(self, data, exclude, compression)

    def send_to_node(self, n, data, compression="none"):
        self._net._send_to_node(self, n, data, compression)

    # -- lifecycle: no sockets, no threads -----------------------------------------------------
    def start(self):
        pass

    def join(self, timeout=None):
        pass

    def stop(self):
        self.node_request_to_stop()
        self.terminate_flag.set()

    def connect_with_node(self, host, port, reconnect=False):
        """Dial another simulated node (node.py:122-176): self connections are refused, an
        existing connection is reported; the new connection exists from the next round on
        (its connected events fire then, like the reference's asynchronous handshake)."""
        if host == self.host and port == self.port:
            print("connect_with_node: Cannot connect with yourself!!")
            return False
        peer = self._net._peer_at(host, port)
        if peer is None:
            self.outbound_node_connection_error(ConnectionRefusedError(f"{host}:{port}"))
            return False
        if peer in self._net._conn[self._peer] or self._net._queued(self._peer, peer, True):
            self.debug_print(f"connect_with_node: Already connected with this node ({host}:{port}).")
            return True
        self._net._queue_change(self._peer, peer, True)
        return True

    def disconnect_with_node(self, node):
        """Close one of our outbound connections (node.py:178-189); it goes away between rounds
        -- messages in flight on it are lost -- and both ends see node_disconnected."""
        if node in self.nodes_outbound:
            self.node_disconnect_with_outbound_node(node)
            node.stop()
            self._net._queue_change(self._peer, node.peer, False)
        else:
            self.debug_print("Node disconnect_with_node: cannot disconnect with a node with which we are not connected.")

    # -- event hooks (node.py:282-363), identical callback dispatch ----------------------------
    def outbound_node_connected(self, node):
        self.debug_print(f"outbound_node_connected: {node.id}")
        if self.callback is not None:
            self.callback("outbound_node_connected", self, node, {})

    def outbound_node_connection_error(self, exception):
        self.debug_print(f"outbound_node_connection_error: {exception}")
        if self.callback is not None:
            self.callback("outbound_node_connection_error", self, None, {"exception": exception})

    def inbound_node_connected(self, node):
        self.debug_print(f"inbound_node_connected: {node.id}")
        if self.callback is not None:
            self.callback("inbound_node_connected", self, node, {})

    def inbound_node_connection_error(self, exception):
        self.debug_print(f"inbound_node_connection_error: {exception}")
        if self.callback is not None:
            self.callback("inbound_node_connection_error", self, None, {"exception": exception})

    def node_disconnected(self, node):
        if node in self.nodes_inbound:
            del self.nodes_inbound[self.nodes_inbound.index(node)]
            self.inbound_node_disconnected(node)
        if node in self.nodes_outbound:
            del self.nodes_outbound[self.nodes_outbound.index(node)]
            self.outbound_node_disconnected(node)

    def inbound_node_disconnected(self, node):
        self.debug_print(f"inbound_node_disconnected: {node.id}")
        if self.callback is not None:
            self.callback("inbound_node_disconnected", self, node, {})

    def outbound_node_disconnected(self, node):
        self.debug_print(f"outbound_node_disconnected: {node.id}")
        if self.callback is not None:
            self.callback("outbound_node_disconnected", self, node, {})

    def node_message(self, node, data):
        self.debug_print(f"node_message: {node.id}: {data}")
        if self.callback is not None:
            self.callback("node_message", self, node, data)

    def node_disconnect_with_outbound_node(self, node):
        self.debug_print(f"node wants to disconnect with other outbound node: {node.id}")
        if self.callback is not None:
            self.callback("node_disconnect_with_outbound_node", self, node, {})

    def node_request_to_stop(self):
        self.debug_print("node is requested to stop!")
        if self.callback is not None:
            self.callback("node_request_to_stop", self, {}, {})

    def node_reconnection_error(self, host, port, trials):
        return True

    def __str__(self):
        return f"Node: {self.host}:{self.port}"

    def __repr__(self):
        return f"<Node {self.host}:{self.port} id: {self.id}>"


class CompatNetwork:
    """A population of ``node_class`` instances over ``graph``, relayed by the HIP engine."""

    def __init__(self, graph, node_class=SimNode, mode="flood", fanout=3, host="127.0.0.1",
                 base_port=10000, node_kwargs=None, engine_factory=None, **engine_kw):
        from .network import GraphNetwork
        self.graph, self.mode, self.fanout = graph, mode, int(fanout)
        V = graph.V
        kw = dict(node_kwargs or {})
        self.nodes = []
        for v in range(V):
            n = node_class(host, base_port + v, str(v), **kw)
            n._net, n._peer = self, v
            self.nodes.append(n)
        self._conn = [dict() for _ in range(V)]   # _conn[v][u] = v's connection to u
        rp, ci = graph.rowptr, graph.colidx
        for a in range(V):
            for b in ci[rp[a]:rp[a + 1]]:
                b = int(b)
                if b <= a:
                    continue
                na, nb = self.nodes[a], self.nodes[b]
                ca = SimConnection(na, b, nb.id, nb.host, nb.port)
                cb = SimConnection(nb, a, na.id, na.host, na.port)
                na.nodes_outbound.append(ca)
                nb.nodes_inbound.append(cb)
                self._conn[a][b], self._conn[b][a] = ca, cb
                na.outbound_node_connected(ca)
                nb.inbound_node_connected(cb)
        self._deg = graph.degree()
        self._by_addr = {(n.host, n.port): v for v, n in enumerate(self.nodes)}
        self._changes = []  # (a, b, connect) queued by connect_with_node / disconnect_with_node
        make = engine_factory or GraphNetwork
        self.engine = make(graph, mode=mode, fanout=fanout, **engine_kw)
        self.origins, self.payloads = [], []
        self.absorbed_sends = 0
        self.current_round = -1
        self._dispatching = None  # (node, msg) while a node_message call runs

    # -- sends from app code ----------------------------------------------------------------
    def _originate(self, node, data, compression):
        if node._net is not self:
            raise ValueError("node does not belong to this CompatNetwork")
        ok, obj = wire.round_trip(data, compression=compression)
        if ok:
            self.origins.append(node._peer)
            self.payloads.append(obj)
        else:  # nothing reaches the wire, but node.py:116 has counted every attempt
            node.message_count_send += len(node.all_nodes)

    def _send_to_nodes(self, node, data, exclude, compression):
        if self._dispatching is not None:
            self.absorbed_sends += 1  # the engine already relayed this delivery
            return
        if exclude:
            raise NotImplementedError("compat mode: a broadcast originates to every connection")
        self._originate(node, data, compression)

    def _send_to_node(self, node, conn, data, compression):
        if self._dispatching is not None:
            self.absorbed_sends += 1
            return
        raise NotImplementedError("compat mode: single-connection sends outside a delivery are not "
                                  "broadcasts; use send_to_nodes")

    def _conn_send(self, node, conn, data, compression):
        self._send_to_node(node, conn, data, compression)

    # -- connection changes (applied between rounds) -----------------------------------------
    def _peer_at(self, host, port):
        return self._by_addr.get((host, port))

    def _queued(self, a, b, connect):
        return any({x, y} == {a, b} and c == connect for x, y, c in self._changes)

    def _queue_change(self, a, b, connect):
        self._changes.append((int(a), int(b), bool(connect)))

    def _apply_changes(self):
        """Hand the queued changes to the engine (p2pg_update_edges) and mirror them on the
        node objects: new SimConnections + connected events (dialler outbound, other end
        inbound), removed ones + node_disconnected on both ends (node.py:307-319)."""
        if not self._changes:
            return
        changes, self._changes = self._changes, []
        add = [(a, b) for a, b, c in changes if c]
        rem = [(a, b) for a, b, c in changes if not c]
        self.engine.update_edges(add=add, remove=rem)
        self.graph = self.engine.graph
        self._deg = self.graph.degree()
        for a, b in rem:
            ca, cb = self._conn[a].pop(b), self._conn[b].pop(a)
            self.nodes[a].node_disconnected(ca)
            self.nodes[b].node_disconnected(cb)
        for a, b in add:
            na, nb = self.nodes[a], self.nodes[b]
            ca = SimConnection(na, b, nb.id, nb.host, nb.port)
            cb = SimConnection(nb, a, na.id, na.host, na.port)
            na.nodes_outbound.append(ca)
            nb.nodes_inbound.append(cb)
            self._conn[a][b], self._conn[b][a] = ca, cb
            na.outbound_node_connected(ca)
            nb.inbound_node_connected(cb)

    # -- running ------------------------------------------------------------------------------
    def run(self, max_rounds=1 << 20):
        """Relay every broadcast originated so far to quiescence, dispatching hooks per round.
        Returns the engine's per-round stats."""
        self._apply_changes()  # changes made before the run: the starting topology
        if not self.origins:
            return []
        src = np.asarray(self.origins, dtype=np.int32)
        self.engine.broadcast(src)
        out = []
        k = self.fanout
        while len(out) < max_rounds:
            st = self.engine.step()
            out.append(st)
            self.current_round = st.round
            if st.new_deliveries:
                d = self.engine.deliveries()
                order = np.lexsort((d.msg, d.peer))
                for i in order:
                    self._deliver(int(d.peer[i]), int(d.msg[i]), int(d.parent[i]), st.round, k)
            self.between_rounds(st.round)
            self._apply_changes()  # made by the hooks of this round: effective from the next
            if not st.active:
                break
        return out

    def between_rounds(self, rnd):
        """Called after round rnd's node_message calls, before queued connection changes are
        applied (override to drive topology changes from outside the nodes)."""

    def _deliver(self, v, m, parent, rnd, k):
        node = self.nodes[v]
        deg = int(self._deg[v])
        if self.mode == "gossip":
            node.message_count_send += min(k, deg)
        else:
            node.message_count_send += deg if rnd == 0 else max(deg - 1, 0)
        if rnd == 0:
            return  # the origin's own send_to_nodes call; no node_message at the origin
        node.message_count_recv += 1
        self._dispatching = (node, m)
        try:
            node.node_message(self._conn[v][parent], self.payloads[m])
        finally:
            self._dispatching = None

    def close(self):
        self.engine.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
