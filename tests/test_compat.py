"""Per-callback compat mode (p2pnetwork.gpu.compat): a Node-style dedup-relay app, written
against the reference's hook surface, runs unchanged on CompatNetwork and reproduces the
golden fixtures made with the reference's own Node objects (first-receipt round and sender per
peer and message, total relays = sum of message_count_send).  CPU tests drive it with the
test-only engine stand-in (tests/partition_mock.py); the gpu-marked ones with the HIP engine."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden, updates_of
from partition_mock import MockEngine


def dedup_app():
    from p2pnetwork.gpu.compat import SimNode

    class DedupRelay(SimNode):  # the app of README.md:20 / examples, unchanged in shape
        def __init__(self, host, port, id=None, callback=None, max_connections=0):
            super().__init__(host, port, id, callback, max_connections)
            self.seen = {}

        def node_message(self, node, data):
            mid = data["mid"]
            if mid in self.seen:
                return
            self.seen[mid] = (self._net.current_round, int(node.id))
            self.send_to_nodes(data, exclude=[node])

    return DedupRelay


def run_compat(z, factory=None):
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.compat import CompatNetwork
    g = PeerGraph(z["rowptr"], z["colidx"])
    kw = dict(mode=str(z["mode"]), fanout=int(z["fanout"]), gossip_seed=int(z["gossip_seed"]),
              churn_threshold_value=int(z["churn_threshold"]), churn_seed=int(z["churn_seed"]))
    if factory is not None:
        kw["engine_factory"] = factory
    net = CompatNetwork(g, dedup_app(), **kw)
    for m, s in enumerate(z["src"]):
        net.nodes[int(s)].seen[m] = (0, -1)
        net.nodes[int(s)].send_to_nodes({"mid": m})
    net.run()
    V, M = g.V, len(z["src"])
    hop = np.full((V, M), -1, np.int32)
    par = np.full((V, M), -1, np.int32)
    for v, n in enumerate(net.nodes):
        for m, (h, p) in n.seen.items():
            hop[v, m], par[v, m] = h, p
    sends = sum(n.message_count_send for n in net.nodes)
    recv = sum(n.message_count_recv for n in net.nodes)
    net.close()
    return hop, par, sends, recv, net


def check(z, hop, par, sends, recv):
    np.testing.assert_array_equal(hop, z["hop"])
    np.testing.assert_array_equal(par, z["parent"])
    assert sends == int(z["round_relays"].sum())
    assert recv == int((z["hop"] > 0).sum())  # first receipts (the origin gets no node_message)


@pytest.mark.parametrize("name", golden_cases())
def test_compat_mock_engine_matches_reference_golden(name):
    z = load_golden(name)
    hop, par, sends, recv, _ = run_compat(z, MockEngine)
    check(z, hop, par, sends, recv)


def test_compat_lifecycle_and_payload_codec():
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.compat import CompatNetwork, SimNode
    events = []

    def cb(event, main_node, connected_node, data):
        events.append((event, main_node.id, getattr(connected_node, "id", None), data))

    g = PeerGraph.from_edges(4, [(0, 1), (1, 2), (2, 3)])
    net = CompatNetwork(g, SimNode, node_kwargs={"callback": cb}, engine_factory=MockEngine)
    assert [e[:3] for e in events] == [
        ("outbound_node_connected", "0", "1"), ("inbound_node_connected", "1", "0"),
        ("outbound_node_connected", "1", "2"), ("inbound_node_connected", "2", "1"),
        ("outbound_node_connected", "2", "3"), ("inbound_node_connected", "3", "2")]
    assert [c.id for c in net.nodes[1].all_nodes] == ["0", "2"]
    events.clear()
    net.nodes[0].send_to_nodes({"t": (1, 2)})   # tuple -> list through the JSON codec
    net.nodes[3].send_to_nodes("42")             # a str holding JSON arrives parsed
    net.nodes[3].send_to_nodes(12345)            # not sendable: counted, reaches nobody
    net.run()
    got = [(e[1], e[2], e[3]) for e in events if e[0] == "node_message"]
    # round 1: peer 1 gets msg 0 from 0, peer 2 gets msg 1 from 3; round 2: 2<-1 (m0), 1<-2 (m1)
    assert got == [("1", "0", {"t": [1, 2]}), ("2", "3", 42), ("1", "2", 42), ("2", "1", {"t": [1, 2]}),
                   ("0", "1", 42), ("3", "2", {"t": [1, 2]})]
    # flood relays: origin deg, others deg-1; the unsendable send counted 1 at peer 3
    assert [n.message_count_send for n in net.nodes] == [1, 2, 2, 1 + 1]
    assert [n.message_count_recv for n in net.nodes] == [1, 2, 2, 1]
    net.nodes[2].stop()
    assert events[-1][0] == "node_request_to_stop"


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_cases())
def test_compat_gpu_engine_matches_reference_golden(name):
    z = load_golden(name)
    hop, par, sends, recv, net = run_compat(z)
    check(z, hop, par, sends, recv)
    assert net.absorbed_sends == recv if str(z["mode"]) == "flood" else True


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_cases(dynamic=True))
def test_compat_gpu_connection_changes_match_reference_golden(name):
    """Node-style connect_with_node / disconnect_with_node between rounds (the dialler is the
    lower id, as in the reference harness) reproduce the dyn_* fixtures; the lifecycle events
    fire on both ends."""
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.compat import CompatNetwork
    z = load_golden(name)
    upd = updates_of(z)
    events = []

    class Net(CompatNetwork):
        def between_rounds(self, rnd):
            if rnd not in upd:
                return
            add, rem = upd[rnd]
            for a, b in rem:
                a, b = sorted((int(a), int(b)))
                self.nodes[a].disconnect_with_node(self.connection(a, b))
            for a, b in add:
                a, b = sorted((int(a), int(b)))
                assert self.nodes[a].connect_with_node(self.nodes[b].host, self.nodes[b].port)

    def cb(event, main_node, connected_node, data):
        if event != "node_message":
            events.append(event)

    App = dedup_app()
    g = PeerGraph(z["rowptr"], z["colidx"])
    net = Net(g, App, mode=str(z["mode"]), fanout=int(z["fanout"]), gossip_seed=int(z["gossip_seed"]),
              churn_threshold_value=int(z["churn_threshold"]), churn_seed=int(z["churn_seed"]),
              node_kwargs={"callback": cb})
    events.clear()
    for m, s in enumerate(z["src"]):
        net.nodes[int(s)].seen[m] = (0, -1)
        net.nodes[int(s)].send_to_nodes({"mid": m})
    net.run()
    V, M = g.V, len(z["src"])
    hop = np.full((V, M), -1, np.int32)
    par = np.full((V, M), -1, np.int32)
    for v, n in enumerate(net.nodes):
        for m, (h, p) in n.seen.items():
            hop[v, m], par[v, m] = h, p
    check(z, hop, par, sum(n.message_count_send for n in net.nodes), sum(n.message_count_recv for n in net.nodes))
    n_add = sum(len(a) for a, _ in upd.values())
    n_rem = sum(len(r) for _, r in upd.values())
    assert events.count("outbound_node_connected") == events.count("inbound_node_connected") == n_add
    assert events.count("outbound_node_disconnected") == events.count("inbound_node_disconnected") == n_rem
    assert events.count("node_disconnect_with_outbound_node") == n_rem
    net.close()


def test_compat_second_run_relays_only_new_broadcasts():
    """run() relays the broadcasts queued since the previous run(): nothing is replayed, so no
    node_message fires twice for one payload and the counters are not double-counted."""
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.compat import CompatNetwork
    got = []

    class App(dedup_app()):
        def node_message(self, node, data):
            got.append((self.id, data["mid"]))
            super().node_message(node, data)

    g = PeerGraph.from_edges(5, [(0, 1), (1, 2), (2, 3), (3, 4)])
    net = CompatNetwork(g, App, engine_factory=MockEngine)
    net.nodes[0].seen["a"] = (0, -1)
    net.nodes[0].send_to_nodes({"mid": "a"})
    net.run()
    first = list(got)
    assert sorted(first) == [("1", "a"), ("2", "a"), ("3", "a"), ("4", "a")]
    sends = [n.message_count_send for n in net.nodes]
    assert net.run() == []  # nothing new queued: nothing relayed
    net.nodes[4].seen["b"] = (0, -1)
    net.nodes[4].send_to_nodes({"mid": "b"})
    net.run()
    assert sorted(got[len(first):]) == [("0", "b"), ("1", "b"), ("2", "b"), ("3", "b")]
    # second run: flood relays deg at the origin (4: 1), deg-1 elsewhere (1, 1, 1, 0)
    assert [n.message_count_send - s for n, s in zip(net.nodes, sends)] == [0, 1, 1, 1, 1]


def test_compat_repeated_disconnect_is_queued_once():
    """Dropping the same connection twice in one round (e.g. from two node_message calls) is
    harmless, as in the reference: one engine update, both ends see one disconnect."""
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.compat import CompatNetwork, SimNode
    events = []

    def cb(event, main_node, connected_node, data):
        events.append((event, main_node.id))

    class Eng(MockEngine):
        updates = []

        def update_edges(self, add=(), remove=()):
            Eng.updates.append((list(add), list(remove)))
            self.graph = self.g = self.g.with_changes(add, remove)

    g = PeerGraph.from_edges(3, [(0, 1), (1, 2)])
    net = CompatNetwork(g, SimNode, node_kwargs={"callback": cb}, engine_factory=Eng)
    c = net.connection(0, 1)
    net.nodes[0].disconnect_with_node(c)
    net.nodes[0].disconnect_with_node(c)
    # disconnect + connect back in the same round cancel out
    net.nodes[1].disconnect_with_node(net.connection(1, 2))
    assert net.nodes[1].connect_with_node(net.nodes[2].host, net.nodes[2].port)
    net._apply_changes()
    assert Eng.updates == [([], [(0, 1)])]
    assert events.count(("inbound_node_disconnected", "1")) == 1
    assert events.count(("outbound_node_disconnected", "0")) == 1
    assert [c.id for c in net.nodes[1].all_nodes] == ["2"]


def test_compat_higher_id_dialler_is_the_outbound_end():
    """Peer 5 dials peer 2 (connect_with_node, node.py:122-176): 5 holds the outbound handle and
    sees outbound_node_connected, 2 the inbound one -- whatever the id order -- and 5 can later
    close it with disconnect_with_node (it is in 5's nodes_outbound, node.py:178-189)."""
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.compat import CompatNetwork, SimNode
    events = []

    def cb(event, main_node, connected_node, data):
        events.append((event, main_node.id, getattr(connected_node, "id", None)))

    class Eng(MockEngine):
        updates = []

        def update_edges(self, add=(), remove=()):
            Eng.updates.append((list(add), list(remove)))
            self.graph = self.g = self.g.with_changes(add, remove)

    g = PeerGraph.from_edges(6, [(0, 1), (1, 2), (3, 4)])
    net = CompatNetwork(g, SimNode, node_kwargs={"callback": cb}, engine_factory=Eng)
    events.clear()
    n2, n5 = net.nodes[2], net.nodes[5]
    assert n5.connect_with_node(n2.host, n2.port)
    net._apply_changes()
    assert events == [("outbound_node_connected", "5", "2"), ("inbound_node_connected", "2", "5")]
    assert [c.id for c in n5.nodes_outbound] == ["2"] and n5.nodes_inbound == []
    assert [c.id for c in n2.nodes_inbound] == ["1", "5"]
    events.clear()
    n5.disconnect_with_node(n5.nodes_outbound[0])
    net._apply_changes()
    assert Eng.updates[-1] == ([], [(2, 5)])
    assert ("node_disconnect_with_outbound_node", "5", "2") in events
    assert ("outbound_node_disconnected", "5", "2") in events
    assert ("inbound_node_disconnected", "2", "5") in events
    assert n5.all_nodes == [] and [c.id for c in n2.all_nodes] == ["1"]
