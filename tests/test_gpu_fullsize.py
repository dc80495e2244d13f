"""Full-size GPU parity at BASELINE.json configurations, through the C-ABI.

* Config 5 -- 100M-peer Watts-Strogatz k=8 beta=0.1, per-round edge-drop churn p=0.05, 4096
  concurrent floods -- unpartitioned on ONE MI355X (seen + two frontier planes = 154 GB of
  its 288 GB).  Checked: the relay identity over the whole seen plane (word by word, never a
  51 GB host copy: p2pg_read_seen_word), reset determinism, words 0 and 63 of the 4096-run ==
  the matching 64-broadcast runs, word 63 == the C oracle's delivered set and per-round
  counters, and word 0's hop / parent planes == the C oracle's bit for bit (100M x 64).
  Reference anchor: the relay of node.py:106-120 with the lost sends of
  nodeconnection.py:123-126.
* A 1M-peer Barabasi-Albert m=4 push-gossip with 4096 broadcasts (all 64 words through the
  packed-E / fused / compact-flush paths): the whole seen plane and every per-round counter ==
  the C oracle, in every push form.
Each test prints nothing for up to ~2 minutes (graph generation and the CPU oracle)."""
import os
from types import SimpleNamespace

import numpy as np
import pytest

from oracle import coracle
from test_gpu_parity import assert_rounds_equal
from test_gpu_partition import _assert_same_rounds

pytestmark = pytest.mark.gpu

CSEED, GSEED = 0xC0FFEE, 0x5EED  # bench.py's seeds


@pytest.fixture(scope="module")
def config5():
    from p2pnetwork.gpu import PeerGraph, make_sources
    from p2pnetwork.gpu.network import churn_threshold
    g = PeerGraph.watts_strogatz(100_000_000, 8, 0.1, seed=1)
    return g, make_sources(g.V, 4096, seed=1), churn_threshold(0.05)


def c5_net(g, thr, **kw):
    from p2pnetwork.gpu import GraphNetwork
    return GraphNetwork(g, mode="flood", churn_threshold_value=thr, churn_seed=CSEED, **kw)


# Config 5's own form is the 1-D vertex partition (BASELINE.json configs[4]).  Two ranks are what
# one MI355X holds at the full 100M peers: each owns 50M peers and keeps 16.7M ghosts, i.e. 66.7M
# rows x 512 B x 3 planes + 2 x 16.7M x 65 int64 of record buffers = 122 GB per rank.
C5_WORLD = 2


def _digest(a):
    import xxhash
    return xxhash.xxh3_128_digest(np.ascontiguousarray(a))


@pytest.fixture(scope="module")
def config5_run(config5):
    """Config 5's 4096-flood run on one engine (then reset and run again): per-round counters,
    |seen set| per peer, words 0 and 63, and a 128-bit digest of every word column over each
    rank's owned range of the C5_WORLD-rank vertex partition (the partitioned run is held to
    those).  The whole plane never comes to the host (51 GB): one word column at a time."""
    from p2pnetwork.gpu.partition import VertexPartition
    g, src, thr = config5
    bounds = VertexPartition.ranges(g, C5_WORLD)
    with c5_net(g, thr) as net:
        net.broadcast(src)
        a = net.run()
        pop = np.zeros(g.V, dtype=np.int64)  # |seen set| per peer, 64 words at a time
        cols, dig, whole = {}, {}, {}
        for w in range(len(src) // 64):
            col = net.seen_word(w)
            pop += np.bitwise_count(col)
            whole[w] = _digest(col)
            for q in range(C5_WORLD):
                dig[w, q] = _digest(col[bounds[q]:bounds[q + 1]])
            if w in (0, 63):
                cols[w] = col
            del col
        net.reset()
        b = net.run()
    return dict(rounds=a, rounds_again=b, pop=pop, cols=cols, dig=dig, whole=whole, bounds=bounds)


def _c5_partitioned(g, src, thr, per_rank, record=False):
    """Config 5 as a C5_WORLD-rank vertex partition: real engines as threads on the one GPU,
    records moved between them by device copies (ThreadTransport), the engine streams waiting
    for the copies (PartitionedNetwork._ready), the next round's interior peers overlapping the
    exchange.  per_rank(rank, net, rounds) runs in the rank's thread before its engine closes."""
    import threading
    from p2pnetwork.gpu import PartitionedNetwork
    from test_gpu_partition import ThreadTransport
    shared = {"slots": [None] * C5_WORLD, "barrier": threading.Barrier(C5_WORLD)}
    out, errors = [None] * C5_WORLD, []

    def rank_main(rank):
        try:
            net = PartitionedNetwork(g, C5_WORLD, rank, ThreadTransport(shared, rank), mode="flood",
                                     churn_threshold_value=thr, churn_seed=CSEED, record=record)
            with net.net:
                net.broadcast(src)
                rounds = net.run()
                out[rank] = per_rank(rank, net, rounds)
        except BaseException as exc:  # surface in the main thread; unblock the other rank
            errors.append(exc)
            shared["barrier"].abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(C5_WORLD)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=800)
    stuck = [r for r, t in enumerate(th) if t.is_alive()]
    if stuck:
        shared["barrier"].abort()  # unblock the other rank; the stuck engine cannot be closed here
        raise AssertionError(f"rank(s) {stuck} of the {C5_WORLD}-rank partition did not finish in 800 s")
    if errors:
        raise errors[0]
    return out


@pytest.mark.timeout(900)
def test_config5_vertex_partitioned_full_size(config5, config5_run):
    """Config 5 in its own form: 100M-peer WS k=8 beta=0.1, churn 0.05, 4096 floods, vertex-
    partitioned over 2 ranks (50M owned + 16.7M ghost rows each; records of 1 + 64 int64 per live
    boundary row, list segments, >= 2^30-word record buffers) -- every owned word column of every
    rank == the one-engine run's (digest per word and rank range), every global per-round counter
    == the one-engine run's.  Anchors: the relay node.py:106-120 with the lost sends of
    nodeconnection.py:123-126; the cross-host fan-out it replaces, nodeconnection.py:107-160."""
    g, src, thr = config5
    ref = config5_run
    M = len(src)

    def check(rank, net, rounds):
        p = net.part
        assert p.lo == ref["bounds"][rank] and p.hi == ref["bounds"][rank + 1]
        assert p.V_local > 60_000_000 and len(p.send_local) * (1 + M // 64) > 1 << 30
        bad = []
        own = p.owned_local
        buf = np.empty(len(own), dtype=np.uint64)
        for w in range(M // 64):
            np.take(net.net.seen_word(w), own, out=buf)
            if _digest(buf) != ref["dig"][w, rank]:
                bad.append(w)
            if w == 0 and rank == 0:  # one column exactly, not only by digest
                np.testing.assert_array_equal(buf, ref["cols"][0][p.lo:p.hi])
        return rounds, bad, [r.push_form for r in net.local_rounds]

    res = _c5_partitioned(g, src, thr, check)
    for rank, (rounds, bad, _) in enumerate(res):
        assert not bad, f"rank {rank}: owned seen words {bad} differ from the one-engine run"
        _assert_same_rounds(rounds, ref["rounds"])  # global counters, every round


def test_config5_full_size_flood_churn(config5, config5_run):
    g, src, thr = config5
    M = len(src)
    deg = g.degree()
    a, b, pop, cols = (config5_run[k] for k in ("rounds", "rounds_again", "pop", "cols"))
    assert [r.as_dict() for r in a] == [r.as_dict() for r in b]
    delivered = int(pop.sum())
    assert delivered == sum(r.new_deliveries for r in a)
    assert 0.99 * g.V * M < delivered <= g.V * M  # churn loses sends, not (on WS) whole peers
    # every first receipt relays deg - 1 (the sender excluded), the origin deg: node.py:106-116
    assert sum(r.relays for r in a) == int((pop * (deg - 1)).sum()) + M
    for w, col in cols.items():
        with c5_net(g, thr, msg_id_base=64 * w) as sub:
            sub.broadcast(src[64 * w:64 * w + 64])
            rounds = sub.run()
            np.testing.assert_array_equal(sub.seen_word(0), col)
    ora = coracle.run(g.rowptr, g.colidx, src[64 * 63:], "flood", churn_threshold=thr,
                      churn_seed=CSEED, record=False, want_seen=True)
    np.testing.assert_array_equal(ora.seen[:, 0], cols[63])
    assert_rounds_equal(rounds, ora.rounds)


def test_config5_full_size_every_word_matches_oracle_digests(config5, config5_run):
    """All 64 words of config 5's 4096-flood seen plane (100M peers, churn 0.05) == the C
    oracle's 64-flood runs of their messages, which re-draw every churn decision (128-bit
    digests made in the build container), and the additive per-round counters == the sums --
    the whole plane pinned to the oracle in the default suite (node.py:106-120 with the lost
    sends of nodeconnection.py:123-126).  Since the partitioned run is held to the same
    per-rank digests of these columns above, it is pinned to the oracle too."""
    from test_gpu_parity import assert_plane_matches_digests, plane_fixture
    g, src, _ = config5
    z = plane_fixture("plane_c5_ws100m_churn")
    assert int(z["V"]) == g.V and int(z["M"]) == len(src)
    whole = config5_run["whole"]  # the column digests taken as the plane was read
    assert_plane_matches_digests(z, g, lambda w: np.frombuffer(whole[w], dtype=np.uint8),
                                 config5_run["rounds"])


def _c5_word_range():
    r = os.environ.get("P2PG_C5_WORDS", "")
    if not r:
        return None
    lo, hi = (int(x) for x in r.split("-"))
    return range(lo, hi + 1)


@pytest.mark.skipif(_c5_word_range() is None,
                    reason="config 5 seen plane vs the C oracle, words lo..hi (~25 s each): P2PG_C5_WORDS=lo-hi")
@pytest.mark.timeout(1500)
def test_config5_full_size_words_match_c_oracle(config5):
    """Words lo..hi of config 5's 4096-flood seen plane (100M peers, churn 0.05) == the C
    oracle's 64-flood runs of their messages, whose every churn decision it re-draws; run in
    ranges (P2PG_C5_WORDS) so that the 64 words fit the box's time limit per call."""
    g, src, thr = config5
    words = _c5_word_range()
    with c5_net(g, thr) as net:
        net.broadcast(src)
        net.run()
        cols = {w: net.seen_word(w) for w in words}
    for w in words:
        ora = coracle.run(g.rowptr, g.colidx, src[64 * w:64 * (w + 1)], "flood", churn_threshold=thr,
                          churn_seed=CSEED, record=False, want_seen=True)
        assert np.array_equal(cols.pop(w), ora.seen[:, 0]), f"word {w}"
        print(f"word {w}: {len(ora.rounds)} rounds, equal", flush=True)
        del ora


def test_config5_word0_hop_parent_match_c_oracle(config5):
    """Messages 0..63 of config 5: first-receipt round and lowest-id surviving sender of all
    100M peers, bit for bit against the C oracle (which re-draws every churn decision) -- on one
    engine, and as the 2-rank vertex partition (every owned row of each rank; parents across the
    rank boundary are ghost senders whose frontier rows arrived as records)."""
    g, src, thr = config5
    with c5_net(g, thr, record=True) as net:
        net.broadcast(src[:64])
        rounds = net.run()
        hop, parent = net.hop_parent()
    ora = coracle.run(g.rowptr, g.colidx, src[:64], "flood", churn_threshold=thr, churn_seed=CSEED,
                      record=True)
    assert_rounds_equal(rounds, ora.rounds)
    assert np.array_equal(hop, ora.hop)
    del hop
    assert np.array_equal(parent, ora.parent)
    del parent

    def check(rank, pnet, prounds):
        p = pnet.part
        h, par = pnet.net.hop_parent()
        own = p.owned_local
        step = 1 << 22
        for a in range(0, len(own), step):  # owned rows in global order, 4M at a time
            rows = own[a:a + step]
            assert np.array_equal(h[rows], ora.hop[p.lo + a:p.lo + a + len(rows)]), f"rank {rank} hop"
            assert np.array_equal(par[rows], ora.parent[p.lo + a:p.lo + a + len(rows)]), f"rank {rank} parent"
        return prounds

    for prounds in _c5_partitioned(g, src[:64], thr, check, record=True):
        _assert_same_rounds(prounds, [SimpleNamespace(**r) for r in ora.rounds])


@pytest.mark.parametrize("push", ["auto", "atomic", "store_unfused"])
def test_gossip_full_width_1m_matches_c_oracle(push, monkeypatch):
    """1M-peer BA m=4, 4096 push-gossips, k=3: the whole seen plane (all 64 words) and every
    per-round counter equal the C oracle's -- auto (dense rounds fused, packed E, compact
    flush), row atomics only, and edge stores with separate pull / scatter passes."""
    from p2pnetwork.gpu import GraphNetwork, PeerGraph, make_sources
    monkeypatch.setenv("P2PG_GOSSIP_PUSH", "auto" if push == "auto" else push.split("_")[0])
    monkeypatch.setenv("P2PG_FUSED", "0" if push == "store_unfused" else "1")
    g = PeerGraph.barabasi_albert(1_000_000, 4, seed=5)
    src = make_sources(g.V, 4096, seed=5)
    with GraphNetwork(g, mode="gossip", fanout=3, gossip_seed=GSEED) as net:
        net.broadcast(src)
        rounds = net.run()
        seen = net.seen_plane()
    forms = {r.push_form for r in rounds if r.new_deliveries}
    if push == "auto":
        assert 3 in forms and 1 in forms, forms  # fused dense rounds and atomic sparse rounds
    ora = coracle.run(g.rowptr, g.colidx, src, "gossip", 3, GSEED, record=False, want_seen=True)
    np.testing.assert_array_equal(seen, ora.seen)
    assert_rounds_equal(rounds, ora.rounds)


def _hub_graph(V, m, seed):
    """Power-law graph plus two stars wider than the pull hub threshold (deg > 512): hub
    senders push through chunk items, hub receivers pull through k_pull_hub_*, and rows of
    64 < deg <= 512 walk their slot words 64 at a time."""
    from p2pnetwork.gpu import PeerGraph
    g = PeerGraph.barabasi_albert(V, m, seed)
    rows = np.repeat(np.arange(g.V), g.degree())
    keep = rows < g.colidx
    e = list(zip(rows[keep].tolist(), g.colidx[keep].tolist()))
    e += [(7, j) for j in range(100, 2100)]
    e += [(V - 1, j) for j in range(0, V - 1, 97)]
    return PeerGraph.from_edges(g.V, e)


@pytest.mark.parametrize("push", ["auto", "store_unfused", "update_push"])
@pytest.mark.parametrize("V,M,fanout,churn", [(200_000, 1500, 3, 0.1), (120_000, 2048, 4, 0.0)])
def test_gossip_wide_rows_hubs_churn_match_c_oracle(V, M, fanout, churn, push, monkeypatch):
    """Rows of 24 and 32 words (W > 16: one peer per wave, packed E rows and slot words) with
    a ragged last word, churn (lost sends leave their slot word empty) and hubs: the whole
    seen plane and every per-round counter == the C oracle, fused and unfused, and with every
    round after a sparse one run as update + E pushes in one pass (P2PG_UPDATE_PUSH=1: touched
    hubs by the hub-only update and atomics)."""
    from p2pnetwork.gpu import GraphNetwork, make_sources
    from p2pnetwork.gpu.network import churn_threshold
    monkeypatch.setenv("P2PG_GOSSIP_PUSH", "auto")
    monkeypatch.setenv("P2PG_FUSED", "0" if push == "store_unfused" else "1")
    monkeypatch.setenv("P2PG_UPDATE_PUSH", "1" if push == "update_push" else "0")
    monkeypatch.setenv("P2PG_V_THRESH", "0.3")  # dense rounds from 30 % active peers on
    g = _hub_graph(V, 4, seed=V + M)
    src = make_sources(g.V, M, seed=7)
    thr = churn_threshold(churn) if churn else 0
    with GraphNetwork(g, mode="gossip", fanout=fanout, gossip_seed=GSEED,
                      churn_threshold_value=thr, churn_seed=CSEED) as net:
        net.broadcast(src)
        rounds = net.run()
        seen = net.seen_plane()
    forms = {r.push_form for r in rounds if r.new_deliveries}
    assert (2 if push == "store_unfused" else 3) in forms, forms  # dense rounds ran
    assert (push == "update_push") == (4 in forms), forms
    ora = coracle.run(g.rowptr, g.colidx, src, "gossip", fanout, GSEED, churn_threshold=thr,
                      churn_seed=CSEED, record=False, want_seen=True)
    np.testing.assert_array_equal(seen, ora.seen)
    assert_rounds_equal(rounds, ora.rounds)


@pytest.mark.parametrize("M", [4096, 512])
def test_run_chunks_keep_the_last_frontier(M, monkeypatch):
    """p2pg_run drops the frontier rows of fused rounds nobody can observe, but the last round a
    call may run keeps them: runs cut after a fused round give the same deliveries and seen
    plane as round-by-round stepping (W = 64: one peer per wave; W = 8: grouped kernel)."""
    from p2pnetwork.gpu import GraphNetwork, PeerGraph, make_sources
    monkeypatch.setenv("P2PG_V_THRESH", "0.3")  # dense rounds from 30 % active peers on
    # (W = 64 on 100K peers: each cut compares a whole round's delivery stream, up to ~10^8 records)
    g = PeerGraph.barabasi_albert(100_000 if M > 512 else 200_000, 4, seed=3)
    src = make_sources(g.V, M, seed=3)
    with GraphNetwork(g, mode="gossip", fanout=3, gossip_seed=GSEED) as a, \
            GraphNetwork(g, mode="gossip", fanout=3, gossip_seed=GSEED) as b:
        a.broadcast(src)
        b.broadcast(src)
        done = 0
        fused_cuts = 0
        for chunk in (9, 2, 3, 1, 4, 50):
            ra = a.run(max_rounds=chunk)
            rb = [b.step() for _ in range(len(ra))]
            assert [r.as_dict() for r in ra] == [r.as_dict() for r in rb]
            done += len(ra)
            fused_cuts += ra[-1].push_form == 3 and ra[-1].new_deliveries > 0
            da, db = a.deliveries(), b.deliveries()
            assert len(da) == ra[-1].new_deliveries
            for f in ("peer", "msg", "hop", "parent"):
                np.testing.assert_array_equal(getattr(da, f), getattr(db, f))
            if not ra[-1].active:
                break
        assert fused_cuts >= 2
        np.testing.assert_array_equal(a.seen_plane(), b.seen_plane())


def test_quiescent_run_after_unstored_fused_round(monkeypatch):
    """p2pg_run to quiescence with every gossip round in edge form (P2PG_GOSSIP_PUSH=store): the
    last round with receipts is fused and, being more than two rounds before max_rounds, does
    not store its frontier; the quiescent round after it has no deliveries and needs no parents,
    so deliveries() is empty (not an error) and a snapshot can be taken."""
    from p2pnetwork.gpu import GraphNetwork, PeerGraph, make_sources
    monkeypatch.setenv("P2PG_GOSSIP_PUSH", "store")
    g = PeerGraph.random_regular(3000, 8, seed=2)
    src = make_sources(g.V, 256, seed=2)
    with GraphNetwork(g, mode="gossip", fanout=3, gossip_seed=GSEED) as a, \
            GraphNetwork(g, mode="gossip", fanout=3, gossip_seed=GSEED) as b:
        a.broadcast(src)
        b.broadcast(src)
        rounds = a.run()
        assert not rounds[-1].active and rounds[-2].push_form == 3 and rounds[-2].new_deliveries > 0
        d = a.deliveries()
        assert len(d) == 0
        assert len(a.snapshot()) > 0
        step = []
        while True:
            step.append(b.step())
            if not step[-1].active:
                break
        assert [r.as_dict() for r in rounds] == [r.as_dict() for r in step]
        np.testing.assert_array_equal(a.seen_plane(), b.seen_plane())


def test_config3_full_size_matches_c_oracle():
    """Config 3 itself (1M-peer G(n,p) mean degree 16, 4096 concurrent floods) against
    oracle/relay_oracle.c at full size: the whole seen plane (all 4096 broadcasts) and every
    per-round counter; then words 0 and 63 as 64-broadcast runs with their global message ids,
    whose first-receipt round and lowest-id sender planes (1M x 64 each) equal the oracle's bit
    for bit and whose seen word equals the 4096-run's.  Anchor: node.py:106-120."""
    from p2pnetwork.gpu import GraphNetwork, PeerGraph, make_sources
    g = PeerGraph.gnp(1_000_000, 16, seed=1)
    src = make_sources(g.V, 4096, seed=1)
    with GraphNetwork(g, mode="flood") as net:
        net.broadcast(src)
        rounds = net.run()
        seen = net.seen_plane()
    ora = coracle.run(g.rowptr, g.colidx, src, "flood", record=False, want_seen=True)
    np.testing.assert_array_equal(seen, ora.seen)
    assert_rounds_equal(rounds, ora.rounds)
    del ora
    for w in (0, 63):
        s64 = src[64 * w:64 * w + 64]
        with GraphNetwork(g, mode="flood", record=True, msg_id_base=64 * w) as sub:
            sub.broadcast(s64)
            r = sub.run()
            hop, par = sub.hop_parent()
            np.testing.assert_array_equal(sub.seen_word(0), seen[:, w])
        o = coracle.run(g.rowptr, g.colidx, s64, "flood", record=True)
        assert_rounds_equal(r, o.rounds)
        assert np.array_equal(hop, o.hop), f"word {w}: hop planes differ"
        assert np.array_equal(par, o.parent), f"word {w}: parent planes differ"
