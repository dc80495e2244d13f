"""The multi-GPU message split of bench.py (--gpus N): rank r runs broadcasts
[r*M/N, (r+1)*M/N) with their global message ids on its own engine.  Broadcasts are independent
bit lanes (each app's seen set is per message id, README.md:20; Node.send_to_nodes relays one
message, node.py:106-112), so the union of the ranks' results must equal the single-engine run
of all M broadcasts bit for bit: every seen word, and every additive per-round counter.  Ranks
run one after the other on cuda:0 (one process, as the driver's N-GPU job runs them side by
side).  Narrow per-rank rows (W = 64/N words) go through the several-peers-per-wave fused
kernel (relay_grouped.hip) for W <= 16 and the one-peer-per-wave kernel for W = 32."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ADDITIVE = ("new_deliveries", "relays", "active_words", "wedges", "scatter_words")


def _run(g, src, base, **kw):
    from p2pnetwork.gpu import GraphNetwork
    with GraphNetwork(g, mode="gossip", fanout=3, gossip_seed=0x5EED, msg_id_base=base, **kw) as net:
        net.broadcast(src)
        rounds = net.run()
        W = (len(src) + 63) // 64
        cols = [net.seen_word(w) for w in range(W)]
    return rounds, cols


def _sum_rounds(parts):
    n = max(len(p) for p in parts)
    return [{k: sum(getattr(p[i], k) for p in parts if i < len(p)) for k in ADDITIVE} for i in range(n)]


def _check_split(g, M, world, churn=0, bounds=None, one=None):
    """one: the single-engine (rounds, seen columns) of these sources, if already run."""
    from p2pnetwork.gpu import make_sources
    src = make_sources(g.V, M, seed=1)
    full, cols = one if one is not None else _run(g, src, 0, churn_threshold_value=churn,
                                                  churn_seed=0xC0FFEE)
    parts = []
    bounds = bounds or [r * M // world for r in range(world + 1)]
    for r in range(len(bounds) - 1):
        lo, hi = bounds[r], bounds[r + 1]
        rounds, rcols = _run(g, src[lo:hi], lo, churn_threshold_value=churn, churn_seed=0xC0FFEE)
        parts.append(rounds)
        for i, c in enumerate(rcols):
            np.testing.assert_array_equal(c, cols[lo // 64 + i], err_msg=f"rank {r} word {i}")
    want = [{k: getattr(x, k) for k in ADDITIVE} for x in full]
    got = _sum_rounds(parts)
    while want and not any(want[-1].values()):
        want.pop()
    while got and not any(got[-1].values()):
        got.pop()
    assert got == want


@pytest.mark.parametrize("world,vthr", [(2, None), (4, None), (8, None), (4, "0.3"), (8, "0.3")])
def test_message_split_union_equals_one_engine_1m(world, vthr, monkeypatch):
    """vthr: the dense-round entry threshold (active peers / V); narrow rows default to 0.95 (few
    dense rounds), 0.3 runs most rounds through the grouped fused kernel."""
    from p2pnetwork.gpu import PeerGraph
    if vthr is not None:
        monkeypatch.setenv("P2PG_V_THRESH", vthr)
    _check_split(PeerGraph.barabasi_albert(1_000_000, 4, seed=3), 4096, world)


def test_message_split_union_with_churn_and_ragged_words():
    """Gossip with churn; M = 2129 split at word boundaries 0 | 1024 | 1984 | 2129 (the last
    rank's last word is partial)."""
    from p2pnetwork.gpu import PeerGraph
    _check_split(PeerGraph.watts_strogatz(200_000, 8, 0.1, seed=4), 2129, 3, churn=200_000_000,
                 bounds=[0, 1024, 1984, 2129])


@pytest.fixture(scope="module")
def c4_one():
    """Config 4's graph and its one-engine run (rounds, 64 seen columns), shared by the three
    split sizes (one graph generation and one reference run instead of three)."""
    from p2pnetwork.gpu import PeerGraph, make_sources
    g = PeerGraph.barabasi_albert(10_000_000, 4, seed=1)
    src = make_sources(g.V, 4096, seed=1)
    return g, _run(g, src, 0, churn_threshold_value=0, churn_seed=0xC0FFEE)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_message_split_config4_full_size(world, c4_one):
    """Config 4 itself (10M-peer BA m=4, 4096 gossips, k=3) as the 2- / 4- / 8-GPU jobs run it:
    the W = 32 / 16 / 8 shares (HALF-mode fused kernel, grouped kernels) union to the one-engine
    run, word for word and counter for counter."""
    g, one = c4_one
    _check_split(g, 4096, world, one=one)
