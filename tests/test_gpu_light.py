"""GPU: light dense gossip rounds (relay_light.hip, k_gossip_light: the low-degree peers one lane
each, the others through k_gossip_fused).  Only the kernel split depends on the round's
lightness, never a result: every fused round taken light (P2PG_LIGHT=1), none (P2PG_LIGHT=0) and
the default rule give identical per-round counters and seen planes, equal to the C oracle, with
and without churn, for fanouts 2 / 3 / 5 (the K = 0 generic-pick instance), and the hop / parent
planes of record mode (whole frontier rows) equal too.  Reference anchor: the relay of first
receipts by Node.send_to_node on the chosen connections (node.py:114-120), lost sends
(nodeconnection.py:123-126)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ("new_deliveries", "relays", "active_vertices", "active_words", "wedges", "deg_active",
          "scatter_words", "touched_words", "received")


def _rows(rounds):
    return [tuple(getattr(r, f) for f in FIELDS) for r in rounds]


def _run(g, src, fanout, thr, light, monkeypatch, record=False):
    from p2pnetwork.gpu import GraphNetwork
    monkeypatch.setenv("P2PG_LIGHT", light)
    with GraphNetwork(g, mode="gossip", fanout=fanout, gossip_seed=0x5EED, churn_threshold_value=thr,
                      churn_seed=0xC0FFEE, record=record) as net:
        net.broadcast(src)
        if record:  # step by step: every frontier row stored whole (store_f == 1)
            rounds = []
            while True:
                st = net.step()
                rounds.append(st)
                if not st.active:
                    break
            return rounds, net.seen_plane(), net.hop_parent()
        return net.run(), net.seen_plane(), None


@pytest.mark.parametrize("fanout,thr", [(3, 0), (3, 200_000_000), (2, 0), (5, 100_000_000)])
def test_light_rounds_change_nothing(fanout, thr, monkeypatch):
    from oracle import coracle
    from p2pnetwork.gpu import PeerGraph, make_sources
    g = PeerGraph.barabasi_albert(400_000, 4, seed=21)
    src = make_sources(g.V, 4096, seed=22)
    ref = _run(g, src, fanout, thr, "0", monkeypatch)
    for light in ("1", "-1"):
        got = _run(g, src, fanout, thr, light, monkeypatch)
        assert _rows(got[0]) == _rows(ref[0]), light
        np.testing.assert_array_equal(got[1], ref[1], err_msg=f"P2PG_LIGHT={light}")
    ora = coracle.run(g.rowptr, g.colidx, src, "gossip", fanout, 0x5EED, 0, thr, 0xC0FFEE, record=False,
                      want_seen=True)
    np.testing.assert_array_equal(ref[1], ora.seen)


@pytest.mark.parametrize("M", [2048, 4096])  # W = 32 / 64
def test_light_rounds_hop_parent_whole_rows(M, monkeypatch):
    from p2pnetwork.gpu import PeerGraph, make_sources
    g = PeerGraph.barabasi_albert(60_000, 3, seed=23)
    src = make_sources(g.V, M, seed=24)
    a = _run(g, src, 3, 150_000_000, "0", monkeypatch, record=True)
    b = _run(g, src, 3, 150_000_000, "1", monkeypatch, record=True)
    assert _rows(a[0]) == _rows(b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2][0], b[2][0])
    np.testing.assert_array_equal(a[2][1], b[2][1])
