"""Per-callback compat mode (p2pnetwork.gpu.compat): Node-style apps, written against the
reference's hook surface, run unchanged on CompatNetwork with the reference's hook semantics --
node_message for every arriving packet, duplicates included (nodeconnection.py:211-216), the
app's own relay decision -- and reproduce fixtures made with the reference's own Node objects:
the dedup relay's first-receipt round and sender per (peer, msg), sum of message_count_send and
of message_count_recv (the fixture's total_recv), and, for apps beyond the dedup relay
(tests/compat_apps.py), every node_message call in order and every node's counters.  CPU tests
drive it with the test-only engine stand-in (tests/partition_mock.py); the gpu-marked ones with
the HIP engine (p2pg_get_sends / p2pg_drop_relays)."""
import json

import numpy as np
import pytest

import compat_apps
from conftest import app_cases, golden_cases, load_golden, updates_of
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


def harness_gossip_app():
    """The fixtures' gossip app as the reference harness writes it (make_golden.py RelayNode):
    send_to_node on the k Philox-chosen connections of a first receipt."""
    from p2pnetwork.gpu.compat import SimNode

    class GossipRelay(SimNode):
        def __init__(self, host, port, id=None, callback=None, max_connections=0):
            super().__init__(host, port, id, callback, max_connections)
            self.seen = {}

        def node_message(self, node, data):
            mid = data["mid"]
            if mid in self.seen:
                return
            self.seen[mid] = (self._net.current_round, int(node.id))
            for c in self._net.gossip_connections(self, mid):
                self.send_to_node(c, data)

    return GossipRelay


def run_compat(z, factory=None, app=None):
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.compat import CompatNetwork
    g = PeerGraph(z["rowptr"], z["colidx"])
    kw = dict(mode=str(z["mode"]), fanout=int(z["fanout"]), gossip_seed=int(z["gossip_seed"]),
              churn_threshold_value=int(z["churn_threshold"]), churn_seed=int(z["churn_seed"]))
    if factory is not None:
        kw["engine_factory"] = factory
    net = CompatNetwork(g, app or dedup_app(), **kw)
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
    # every arriving packet, duplicates included, less the lost sends (nodeconnection.py:215)
    assert recv == int(z["total_recv"])


@pytest.mark.parametrize("name", golden_cases())
def test_compat_mock_engine_matches_reference_golden(name):
    z = load_golden(name)
    hop, par, sends, recv, net = run_compat(z, MockEngine)
    check(z, hop, par, sends, recv)
    assert net.explicit_packets == 0  # the dedup relay is carried by the engine alone


@pytest.mark.parametrize("name", [n for n in golden_cases() if "gossip" in n])
def test_compat_mock_harness_gossip_app_matches_reference_golden(name):
    """The fixtures' own gossip app (send_to_node on the Philox-chosen connections) is
    recognised as the engine's relay on the stand-in engine too."""
    z = load_golden(name)
    hop, par, sends, recv, net = run_compat(z, MockEngine, app=harness_gossip_app())
    check(z, hop, par, sends, recv)
    assert net.explicit_packets == 0


def test_compat_explicit_sends_outside_deliveries():
    """send_to_node outside a delivery is a one-connection origination (node.py:114-120),
    NodeConnection.send is one packet without a counter (nodeconnection.py:107-160), an exclude
    list makes a broadcast explicit, and an empty str packet stops its connection's stream for
    good (the eot_pos > 0 loop, nodeconnection.py:211)."""
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.compat import CompatNetwork, SimNode
    got = []

    class Rec(SimNode):
        def node_message(self, node, data):
            got.append((self.id, node.id, data))

    g = PeerGraph.from_edges(4, [(0, 1), (0, 2), (0, 3)])
    net = CompatNetwork(g, Rec, engine_factory=MockEngine)
    n0 = net.nodes[0]
    n0.send_to_node(net.connection(0, 2), {"p": 1})          # counted, one packet
    net.connection(0, 3).send("raw")                        # not counted
    n0.send_to_nodes({"q": 2}, exclude=[net.connection(0, 1)])  # explicit broadcast to 2, 3
    net.nodes[1].send_to_node(net.connection(1, 0), "")      # empty packet: wedges 1 -> 0
    net.nodes[1].send_to_node(net.connection(1, 0), "after")  # never delivered
    net.run()
    assert got == [("2", "0", {"p": 1}), ("2", "0", {"q": 2}), ("3", "0", "raw"), ("3", "0", {"q": 2})]
    assert [n.message_count_send for n in net.nodes] == [1 + 2, 2, 0, 0]
    assert [n.message_count_recv for n in net.nodes] == [0, 0, 2, 2]
    assert net.explicit_packets == 6


def _run_app(name, factory=None):
    """An app_* fixture's app on CompatNetwork: its node_message events and counters."""
    from p2pnetwork.gpu.compat import CompatNetwork, SimNode
    z = load_golden(name)
    app = str(z["app"])
    log = []
    App = type("App", (compat_apps.APPS[app], SimNode), {"log": log})
    g = compat_apps.make_graph(compat_apps.CASES[name][1])
    np.testing.assert_array_equal(g.colidx, z["colidx"])
    kw = dict(churn_threshold_value=int(z["churn_threshold"]), churn_seed=int(z["churn_seed"]))
    if factory is not None:
        kw["engine_factory"] = factory
    net = CompatNetwork(g, App, **kw)
    for peer, data in json.loads(str(z["origins"])):
        net.nodes[peer].originate(data)
    net.run()
    net.close()
    return z, [json.dumps(list(e)) for e in log], net


def _check_app(z, events, net):
    assert events == list(z["events"])
    np.testing.assert_array_equal([n.message_count_send for n in net.nodes], z["sends"])
    np.testing.assert_array_equal([n.message_count_recv for n in net.nodes], z["recvs"])


@pytest.mark.parametrize("name", app_cases())
def test_compat_apps_mock_engine_match_reference_events(name):
    """Apps beyond the dedup relay (no dedup + ttl, acks back to the sender, relays to every
    connection, relays on the second arrival): every node_message call, in order, and every
    node's counters == the reference's own Node objects'."""
    _check_app(*_run_app(name, MockEngine))


def test_compat_recording_app_gets_one_delivery_per_connection():
    """test_node.py:106-194: path 1-0-2, every node calls send_to_nodes once, the callback only
    records -> exactly 4 node_message events (the fan-out law: one delivery per connection);
    nothing is relayed because the app does not relay."""
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.compat import CompatNetwork, SimNode
    events = []

    def cb(event, main_node, connected_node, data):
        if event == "node_message":
            events.append((main_node.id, connected_node.id, data))

    net = CompatNetwork(PeerGraph.from_edges(3, [(0, 1), (0, 2)]), SimNode, node_kwargs={"callback": cb},
                        engine_factory=MockEngine)
    for i in (0, 1, 2):
        net.nodes[i].send_to_nodes(f"message from {i}")
    net.run()
    assert sorted(events) == [("0", "1", "message from 1"), ("0", "2", "message from 2"),
                              ("1", "0", "message from 0"), ("2", "0", "message from 0")]
    assert [n.message_count_send for n in net.nodes] == [2, 1, 1]
    assert [n.message_count_recv for n in net.nodes] == [2, 1, 1]


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
    # SimNode's node_message only fires the callback (node.py:334-338): one hop, no relay
    assert got == [("1", "0", {"t": [1, 2]}), ("2", "3", 42)]
    # every send_to_node call counted (node.py:116), the unsendable one included
    assert [n.message_count_send for n in net.nodes] == [1, 0, 0, 1 + 1]
    assert [n.message_count_recv for n in net.nodes] == [0, 1, 1, 0]
    net.nodes[2].stop()
    assert events[-1][0] == "node_request_to_stop"


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_cases())
def test_compat_gpu_engine_matches_reference_golden(name):
    z = load_golden(name)
    events = []

    class App(dedup_app()):
        def node_message(self, node, data):
            events.append(1)
            super().node_message(node, data)

    hop, par, sends, recv, net = run_compat(z, app=App)
    check(z, hop, par, sends, recv)
    assert len(events) == recv == int(z["total_recv"])  # one node_message per arrival
    assert net.explicit_packets == 0  # every relay stayed in the engine


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in golden_cases() if "gossip" in n])
def test_compat_gpu_harness_gossip_app_matches_reference_golden(name):
    """The fixtures' own gossip app (send_to_node on the Philox-chosen connections, as the
    reference harness wrote it) is recognised as the engine's relay: no explicit packets."""
    z = load_golden(name)
    hop, par, sends, recv, net = run_compat(z, app=harness_gossip_app())
    check(z, hop, par, sends, recv)
    assert net.explicit_packets == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", app_cases())
def test_compat_apps_gpu_engine_match_reference_events(name):
    """As the mock-engine test, through the HIP engine's sends stream and relay withdrawal."""
    _check_app(*_run_app(name))


@pytest.mark.gpu
def test_compat_gpu_recording_apps():
    """The 4-event law of test_node.py:106-194 on the HIP engine, and the reference's example
    node (examples/MyOwnPeer2PeerNode.py:27-28 only prints) on config 2: every broadcast reaches
    exactly the origin's connections -- sum of deg(origin) deliveries, no relay."""
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.compat import CompatNetwork, SimNode
    events = []

    def cb(event, main_node, connected_node, data):
        if event == "node_message":
            events.append((main_node.id, connected_node.id, data))

    with CompatNetwork(PeerGraph.from_edges(3, [(0, 1), (0, 2)]), SimNode, node_kwargs={"callback": cb}) as net:
        for i in (0, 1, 2):
            net.nodes[i].send_to_nodes(f"message from {i}")
        stats = net.run()
    assert len(events) == 4 and sum(s.received for s in stats) == 4

    class MyOwnPeer2PeerNode(SimNode):
        def node_message(self, node, data):
            events.append(("node_message", self.id, node.id, data))

    z = load_golden("c2_rrg1000_flood")
    g = PeerGraph(z["rowptr"], z["colidx"])
    events.clear()
    with CompatNetwork(g, MyOwnPeer2PeerNode) as net:
        for m, s in enumerate(z["src"]):
            net.nodes[int(s)].send_to_nodes({"mid": m})
        stats = net.run()
        deg = g.degree()
        assert len(events) == int(deg[z["src"]].sum()) == 512
        assert sum(n.message_count_recv for n in net.nodes) == 512
        assert sum(s.received for s in stats) == 512 and net.explicit_packets == 0


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
