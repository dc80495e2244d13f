"""Node apps whose hook behaviour goes beyond the dedup relay, written once against the
reference's Node API and run both on the reference's own Node objects (tests/golden/make_golden.py
``apps``, in the build container) and on ``p2pnetwork.gpu.compat.CompatNetwork``
(tests/test_compat.py).  Every node_message call is logged as (receiver id, sender id, payload),
in call order, so the two runs are compared event for event.

An app class is combined with a Node base class: ``type(name, (App, NodeBase), {})``."""
import json


def fmt(data):
    return json.dumps(data, sort_keys=True) if isinstance(data, (dict, list)) else repr(data)


class Recorder:
    log = None  # the run's event list (set on the combined class)

    def record(self, node, data):
        self.log.append((self.id, node.id, fmt(data)))

    def originate(self, data):
        self.__dict__.setdefault("seen", set()).add(data["mid"])
        self.send_to_nodes(data)


class TtlFlood(Recorder):
    """No dedup: every arrival is forwarded with its ttl decremented, until the ttl runs out
    (a different payload on every hop)."""

    def node_message(self, node, data):
        self.record(node, data)
        if data["ttl"] > 0:
            self.send_to_nodes({"mid": data["mid"], "ttl": data["ttl"] - 1}, exclude=[node])


class EchoDedup(Recorder):
    """The dedup relay, plus an acknowledgement back to the sender of every first receipt
    (send_to_node); acknowledgements are recorded, never forwarded."""

    def node_message(self, node, data):
        self.record(node, data)
        if "ack" in data:
            return
        seen = self.__dict__.setdefault("seen", set())
        if data["mid"] in seen:
            return
        seen.add(data["mid"])
        self.send_to_node(node, {"ack": data["mid"], "by": self.id})
        self.send_to_nodes(data, exclude=[node])


class RelayAllDedup(Recorder):
    """Dedup, but a first receipt goes to every connection, its sender included."""

    def node_message(self, node, data):
        self.record(node, data)
        seen = self.__dict__.setdefault("seen", set())
        if data["mid"] in seen:
            return
        seen.add(data["mid"])
        self.send_to_nodes(data)


class SecondArrival(Recorder):
    """Forwards a message (to all but that sender) when it arrives for the second time."""

    def node_message(self, node, data):
        self.record(node, data)
        n = self.__dict__.setdefault("count", {})
        n[data["mid"]] = n.get(data["mid"], 0) + 1
        if n[data["mid"]] == 2:
            self.send_to_nodes(data, exclude=[node])


APPS = {"ttl": TtlFlood, "echo": EchoDedup, "relayall": RelayAllDedup, "second": SecondArrival}

# fixture name -> (app, graph spec, origins, churn p, churn seed); graph spec = (kind, V, a, b, seed)
CASES = {
    "app_ttl_rrg40": ("ttl", ("rrg", 40, 4, 0, 7), [(0, {"mid": 0, "ttl": 3}), (17, {"mid": 1, "ttl": 2})], 0.0, 0),
    "app_echo_ws60_churn": ("echo", ("ws", 60, 4, 0.2, 8), [(3, {"mid": 0}), (3, {"mid": 1}), (41, {"mid": 2})],
                            0.1, 5),
    "app_relayall_ba50": ("relayall", ("ba", 50, 2, 0, 9), [(0, {"mid": 0}), (49, {"mid": 1})], 0.0, 0),
    "app_second_rrg30": ("second", ("rrg", 30, 4, 0, 10),
                         [(5, {"mid": 0}), (6, {"mid": 0}), (20, {"mid": 1}), (21, {"mid": 1}), (22, {"mid": 1})],
                         0.0, 0),
}


def make_graph(spec, PeerGraph=None):
    if PeerGraph is None:
        from p2pnetwork.gpu import PeerGraph
    kind, V, a, b, seed = spec
    if kind == "rrg":
        return PeerGraph.random_regular(V, a, seed=seed)
    if kind == "ws":
        return PeerGraph.watts_strogatz(V, a, b, seed=seed)
    return PeerGraph.barabasi_albert(V, a, seed=seed)
