"""GPU: connection changes between rounds (p2pg_update_edges) and
snapshot / resume (p2pg_snapshot / p2pg_restore, rank 4).

Topology: the dyn_* fixtures were produced by driving the reference's own Node /
NodeConnection objects through Node.disconnect_with_node / node_disconnected and new
connections between rounds (tests/golden/make_golden.py); the engine must reproduce hop,
parent, delivered set and per-round relays bit for bit, and every byte-model counter of the
oracle, in every push form.  Snapshots: a run interrupted by snapshot -> restore into a fresh
engine continues bit-identically (and equals the uninterrupted run and the oracle)."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden, trim_zeros, updates_of
from oracle import relay_oracle
from p2pnetwork.gpu._lib import P2PGError

pytestmark = pytest.mark.gpu

STAT_KEYS = ("new_deliveries", "relays", "active_vertices", "active_words", "wedges", "deg_active",
             "scatter_words")


def make_net(z, record=True, graph=None):
    from p2pnetwork.gpu import GraphNetwork, PeerGraph
    g = graph if graph is not None else PeerGraph(z["rowptr"], z["colidx"])
    return GraphNetwork(g, mode=str(z["mode"]), fanout=int(z["fanout"]), gossip_seed=int(z["gossip_seed"]),
                        churn_threshold_value=int(z["churn_threshold"]), churn_seed=int(z["churn_seed"]),
                        record=record, count_received=True)


def oracle_of(z, updates=None):
    if str(z["mode"]) == "flood":
        return relay_oracle.flood(z["rowptr"], z["colidx"], z["src"], int(z["churn_threshold"]),
                                  int(z["churn_seed"]), updates=updates)
    return relay_oracle.gossip(z["rowptr"], z["colidx"], z["src"], int(z["fanout"]), int(z["gossip_seed"]),
                               0, int(z["churn_threshold"]), int(z["churn_seed"]), updates=updates)


def run_with_updates(net, updates):
    rounds = []
    while True:
        st = net.step()
        rounds.append(st)
        if st.round in updates:
            net.update_edges(*updates[st.round])
        if not st.active:
            return rounds


def assert_rounds(gpu_rounds, ora_rounds):
    g = [r.as_dict() for r in gpu_rounds]
    o = list(ora_rounds)
    blank = {k: 0 for k in STAT_KEYS}
    for i in range(max(len(g), len(o))):
        a = g[i] if i < len(g) else blank
        b = o[i] if i < len(o) else blank
        for k in STAT_KEYS:
            assert a[k] == b[k], (i, k, a[k], b[k])


@pytest.mark.parametrize("push", ["auto", "atomic", "store"])
@pytest.mark.parametrize("name", golden_cases(dynamic=True))
def test_gpu_topology_updates_match_reference_harness(name, push, monkeypatch):
    z = load_golden(name)
    if str(z["mode"]) == "flood" and push != "auto":
        pytest.skip("push form is a gossip setting")
    monkeypatch.setenv("P2PG_GOSSIP_PUSH", push)
    monkeypatch.setenv("P2PG_E_THRESH", "0.05")
    upd = updates_of(z)
    with make_net(z) as net:
        net.broadcast(z["src"])
        rounds = run_with_updates(net, upd)
        hop, parent = net.hop_parent()
        np.testing.assert_array_equal(hop, z["hop"])
        np.testing.assert_array_equal(parent, z["parent"])
        np.testing.assert_array_equal(net.delivered(), z["hop"] >= 0)
        np.testing.assert_array_equal(trim_zeros([r.relays for r in rounds]), trim_zeros(z["round_relays"]))
        assert net.message_count_send == int(z["round_relays"].sum())
        # arrivals, less the sends in flight on removed connections (and churn's)
        assert sum(r.received for r in rounds) == int(z["total_recv"])
    assert_rounds(rounds, oracle_of(z, upd).rounds)


def test_gpu_topology_update_deliveries_stream_parents():
    """The per-round delivery stream (batched node_message hook) reports the parent of the round
    right after an update on the pre-update connections."""
    z = load_golden("dyn_ba500_gossip_k3")
    upd = updates_of(z)
    with make_net(z, record=False) as net:
        net.broadcast(z["src"])
        while True:
            st = net.step()
            if st.new_deliveries:
                d = net.deliveries()
                np.testing.assert_array_equal(d.hop, st.round)
                np.testing.assert_array_equal(z["hop"][d.peer, d.msg], st.round)
                np.testing.assert_array_equal(z["parent"][d.peer, d.msg], d.parent)
            if st.round in upd:
                net.update_edges(*upd[st.round])
            if not st.active:
                break


def test_gpu_topology_update_errors():
    from p2pnetwork.gpu import GraphNetwork, PeerGraph, make_sources
    g = PeerGraph.random_regular(200, 4, seed=3)
    with GraphNetwork(g, mode="flood") as net:
        net.broadcast(make_sources(g.V, 64, seed=1))
        net.step()
        a, b = 0, int(g.neighbours(0)[0])
        with pytest.raises(P2PGError, match="already exists"):
            net.update_edges(add=[(a, b)])
        with pytest.raises(P2PGError, match="self connection"):
            net.update_edges(add=[(5, 5)])
        c = next(x for x in range(1, 200) if x not in set(g.neighbours(0)))
        with pytest.raises(P2PGError, match="no such connection"):
            net.update_edges(remove=[(0, c)])
        net.update_edges(add=[(0, c)], remove=[(a, b)])
        with pytest.raises(P2PGError, match="one update per round"):
            net.update_edges(remove=[(0, c)])
        assert c in set(net.graph.neighbours(0)) and b not in set(net.graph.neighbours(0))


CASES = ["c2_rrg1000_flood", "ws1000_flood_churn05", "ba1000_gossip_k3", "ba500_gossip_k2_churn10",
         "rrg300_flood_m100_dupsrc"]


@pytest.mark.parametrize("push", ["auto", "store"])
@pytest.mark.parametrize("cut", [1, 3])
@pytest.mark.parametrize("name", CASES)
def test_gpu_snapshot_resume_is_bit_identical(name, cut, push, monkeypatch, tmp_path):
    z = load_golden(name)
    if str(z["mode"]) == "flood" and push != "auto":
        pytest.skip("push form is a gossip setting")
    monkeypatch.setenv("P2PG_GOSSIP_PUSH", push)
    with make_net(z) as net:
        net.broadcast(z["src"])
        first = [net.step() for _ in range(cut)]
        path = tmp_path / "snap.npy"
        net.save_snapshot(path)
        sent = net.message_count_send
        rest = net.run()
        hop_a, par_a = net.hop_parent()
        seen_a = net.seen_plane()
    with make_net(z) as net2:
        net2.broadcast(z["src"])
        net2.load_snapshot(path)
        assert net2.message_count_send == sent
        rest2 = net2.run()
        hop_b, par_b = net2.hop_parent()
        np.testing.assert_array_equal(net2.seen_plane(), seen_a)
        assert net2.message_count_send == int(z["round_relays"].sum())
    assert [r.as_dict() for r in rest] == [r.as_dict() for r in rest2]
    assert sum(r.received for r in first + rest2) == int(z["total_recv"])  # (snapshot v3)
    np.testing.assert_array_equal(hop_a, hop_b)
    np.testing.assert_array_equal(par_a, par_b)
    np.testing.assert_array_equal(hop_b, z["hop"])
    np.testing.assert_array_equal(par_b, z["parent"])
    assert_rounds(first + rest2, oracle_of(z).rounds)


@pytest.mark.parametrize("name", ["ba1000_gossip_k3", "ws1000_flood_churn05"])
def test_gpu_deliveries_after_restore(name):
    """step -> snapshot -> restore -> deliveries: the restored round's own first receipts need
    the frontier of the round before it for their parents, which a snapshot does not hold, so
    the stream refuses that one round (instead of reporting zero or wrong records); from the
    next round on the restored engine streams every round's receipts with the fixture's
    parents, and the decay-phase push state (the last round's receipt count) came back too."""
    z = load_golden(name)
    cut = 4
    with make_net(z, record=False) as net:
        net.broadcast(z["src"])
        for _ in range(cut):
            net.step()
        snap = net.snapshot()
    with make_net(z, record=False) as net2:
        net2.broadcast(z["src"])
        net2.restore(snap)
        with pytest.raises(P2PGError, match="restored"):
            net2.deliveries(cap=1 << 16)
        rounds = []
        while True:
            st = net2.step()
            rounds.append(st)
            d = net2.deliveries()
            assert len(d) == st.new_deliveries
            np.testing.assert_array_equal(z["hop"][d.peer, d.msg], st.round)
            np.testing.assert_array_equal(z["parent"][d.peer, d.msg], d.parent)
            if not st.active:
                break
    assert_rounds(rounds, list(oracle_of(z).rounds)[cut:])


def test_gpu_snapshot_with_topology_updates():
    """Snapshot a dynamic-topology run between updates; the restoring engine loads the graph
    as it is at the snapshot and receives the remaining updates."""
    z = load_golden("dyn_rrg300_flood")
    upd = updates_of(z)
    from p2pnetwork.gpu import PeerGraph
    with make_net(z) as net:
        net.broadcast(z["src"])
        for _ in range(2):  # rounds 0, 1 with the updates after them
            st = net.step()
            net.update_edges(*upd[st.round])
        with pytest.raises(P2PGError, match="before a topology update"):
            net.snapshot()
        st = net.step()  # round 2
        snap = net.snapshot()
        g_now = PeerGraph(net.graph.rowptr, net.graph.colidx)
    with make_net(z, graph=g_now) as net2:
        net2.broadcast(z["src"])
        net2.restore(snap)
        net2.update_edges(*upd[st.round])
        while net2.step().active:
            pass
        hop, parent = net2.hop_parent()
    np.testing.assert_array_equal(hop, z["hop"])
    np.testing.assert_array_equal(parent, z["parent"])


def test_gpu_restore_refuses_other_graph_or_sources():
    from p2pnetwork.gpu import GraphNetwork, PeerGraph, make_sources
    g = PeerGraph.random_regular(300, 6, seed=1)
    src = make_sources(g.V, 64, seed=2)
    with GraphNetwork(g, mode="flood") as net:
        net.broadcast(src)
        net.step()
        snap = net.snapshot()
    with GraphNetwork(g, mode="flood") as other:
        other.broadcast(make_sources(g.V, 64, seed=3))
        with pytest.raises(P2PGError, match="sources differ"):
            other.restore(snap)
    with GraphNetwork(PeerGraph.random_regular(300, 6, seed=9), mode="flood") as other:
        other.broadcast(src)
        with pytest.raises(P2PGError, match="graph differs"):
            other.restore(snap)
    with GraphNetwork(g, mode="gossip") as other:
        other.broadcast(src)
        with pytest.raises(P2PGError, match="configuration differs"):
            other.restore(snap)


@pytest.mark.parametrize("M", [1024, 4096])
def test_gpu_gossip_restore_then_update_edges_wide_rows(M, monkeypatch):
    """A gossip run with packed rows (W = 16 / 64: active-word masks AW, which snapshots do not
    carry) restored into a fresh engine and then changing connections at once: the re-push of the
    last round's sends lists words by AW, so the restore rebuilds it from the frontier rows.
    Equal to the uninterrupted run and to the oracle with the same updates, every push form."""
    from p2pnetwork.gpu import GraphNetwork, PeerGraph, make_sources
    g = PeerGraph.barabasi_albert(3000, 3, seed=31)
    src = make_sources(g.V, M, seed=32)
    rng = np.random.default_rng(5)
    rows = np.repeat(np.arange(g.V), g.degree())
    e = np.stack([rows, g.colidx], 1)
    e = e[e[:, 0] < e[:, 1]]
    rem = e[rng.choice(len(e), 200, replace=False)].astype(np.int32)
    have = set(map(tuple, e.tolist()))
    add = []
    while len(add) < 150:
        a, b = sorted(int(x) for x in rng.integers(0, g.V, 2))
        if a != b and (a, b) not in have and [a, b] not in add:
            add.append([a, b])
    upd = {3: (np.array(add, np.int32), rem)}
    kw = dict(mode="gossip", fanout=2, gossip_seed=77, churn_threshold_value=300000000, churn_seed=9)
    for push in ("auto", "atomic", "store"):
        monkeypatch.setenv("P2PG_GOSSIP_PUSH", push)
        with GraphNetwork(g, record=True, **kw) as net:
            net.broadcast(src)
            ra = run_with_updates(net, upd)
            hop_a, par_a = net.hop_parent()
        with GraphNetwork(g, record=True, **kw) as net:
            net.broadcast(src)
            first = [net.step() for _ in range(4)]  # rounds 0..3; the update follows round 3
            snap = net.snapshot()
        with GraphNetwork(g, record=True, **kw) as net2:
            net2.broadcast(src)
            net2.restore(snap)
            net2.update_edges(*upd[3])
            rest = []
            while True:
                st = net2.step()
                rest.append(st)
                if not st.active:
                    break
            hop_b, par_b = net2.hop_parent()
        np.testing.assert_array_equal(hop_b, hop_a, err_msg=push)
        np.testing.assert_array_equal(par_b, par_a, err_msg=push)
        assert [r.as_dict() for r in first + rest] == [r.as_dict() for r in ra], push
    ora = relay_oracle.gossip(g.rowptr, g.colidx, src, 2, 77, 0, 300000000, 9, updates=upd)
    np.testing.assert_array_equal(hop_a, ora.hop)
    np.testing.assert_array_equal(par_a, ora.parent)
