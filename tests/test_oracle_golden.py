"""Pins the oracle (oracle/relay_oracle.py) against the golden fixtures produced by driving
the reference's own Node / NodeConnection objects (tests/golden/make_golden.py): bit-exact
first-receipt hop, lowest-id parent, delivered set and per-round relay counts (the sum of
Node.message_count_send, p2pnetwork/node.py:116)."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden, tcp_cases, trim_zeros, updates_of
from oracle import relay_oracle


def run_oracle(z, updates=None):
    mode = str(z["mode"])
    if mode == "flood":
        return relay_oracle.flood(z["rowptr"], z["colidx"], z["src"], int(z["churn_threshold"]),
                                  int(z["churn_seed"]), updates=updates)
    return relay_oracle.gossip(z["rowptr"], z["colidx"], z["src"], int(z["fanout"]),
                               int(z["gossip_seed"]), 0, int(z["churn_threshold"]), int(z["churn_seed"]),
                               updates=updates)


@pytest.mark.parametrize("name", golden_cases())
def test_oracle_matches_reference_harness(name):
    z = load_golden(name)
    res = run_oracle(z)
    np.testing.assert_array_equal(res.hop, z["hop"])
    np.testing.assert_array_equal(res.parent, z["parent"])
    relays = [r["relays"] for r in res.rounds]
    np.testing.assert_array_equal(trim_zeros(relays), trim_zeros(z["round_relays"]))
    # every delivery is one node_message that passed dedup; deliveries per round = hop counts
    hop = z["hop"]
    for r in res.rounds:
        assert r["new_deliveries"] == int((hop == r["round"]).sum())


@pytest.mark.parametrize("name", golden_cases(dynamic=True))
def test_oracle_dynamic_topology_matches_reference_harness(name):
    """Connection changes between rounds, driven through the reference's own
    disconnect_with_node / node_disconnected and new NodeConnection pairs: in-flight packets
    on removed connections are lost, later sends use the new connections."""
    z = load_golden(name)
    res = run_oracle(z, updates_of(z))
    np.testing.assert_array_equal(res.hop, z["hop"])
    np.testing.assert_array_equal(res.parent, z["parent"])
    relays = [r["relays"] for r in res.rounds]
    np.testing.assert_array_equal(trim_zeros(relays), trim_zeros(z["round_relays"]))
    # the changes do matter: without them the results differ
    assert not np.array_equal(run_oracle(z).hop, z["hop"])


def test_peergraph_with_changes_matches_oracle():
    """GraphNetwork's host-side topology bookkeeping == the oracle's CSR update."""
    from p2pnetwork.gpu.graph import PeerGraph
    z = load_golden("dyn_rrg300_flood")
    g = PeerGraph(z["rowptr"], z["colidx"])
    rp, ci = z["rowptr"], z["colidx"].astype(np.int64)
    for r, (a, d) in sorted(updates_of(z).items()):
        g = g.with_changes(a, d)
        rp, ci = relay_oracle._apply_changes(rp, ci, a, d)
        np.testing.assert_array_equal(g.rowptr, rp)
        np.testing.assert_array_equal(g.colidx, ci)


def test_config2_relay_identity():
    """1k-peer 8-regular, 64 floods: relays = 64 * (8 + 999 * 7)."""
    z = load_golden("c2_rrg1000_flood")
    assert int(z["round_relays"].sum()) == 64 * (8 + 999 * 7)
    assert (z["hop"] >= 0).all()


def test_config1_tcp_reachability():
    """10 real reference Nodes on localhost TCP: the oracle agrees on reachability and on the
    (timing-free) relay count."""
    z = load_golden("config1_tcp")
    res = relay_oracle.flood(z["rowptr"], z["colidx"], z["src"])
    np.testing.assert_array_equal(res.delivered()[:, 0], z["reached"])
    assert res.total_relays == int(z["relays"]) == 17


@pytest.mark.parametrize("name", tcp_cases())
def test_oracle_matches_real_tcp_runs(name):
    """Every real-TCP fixture (config 1, 48 Nodes x 6 concurrent floods, a small world with
    isolated peers): delivered (peer, msg) set and total relays agree."""
    z = load_golden(name)
    res = relay_oracle.flood(z["rowptr"], z["colidx"], z["src"])
    reached = z["reached"].reshape(len(z["rowptr"]) - 1, -1)
    np.testing.assert_array_equal(res.delivered(), reached)
    assert res.total_relays == int(z["relays"])


@pytest.mark.parametrize("name", golden_cases())
def test_c_oracle_matches_reference_harness_and_numpy_oracle(name):
    from oracle import coracle
    z = load_golden(name)
    mode = str(z["mode"])
    res = coracle.run(z["rowptr"], z["colidx"], z["src"], mode, int(z["fanout"]), int(z["gossip_seed"]), 0,
                      int(z["churn_threshold"]), int(z["churn_seed"]))
    np.testing.assert_array_equal(res.hop, z["hop"])
    np.testing.assert_array_equal(res.parent, z["parent"])
    ref = run_oracle(z)
    assert len(res.rounds) == len(ref.rounds)
    for a, b in zip(res.rounds, ref.rounds):
        assert a == b, (a, b)
