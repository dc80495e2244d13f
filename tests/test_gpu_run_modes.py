"""GPU: the host-side round schedule changes nothing.  p2pg_run enqueues several decay-phase
rounds per host synchronisation (run_decay_batch) and p2pg_step launches a sparse round's push
without reading its counters first when the push form is clear (clearly_sparse, bounded list);
both only decide WHEN the host looks at the counters, so every per-round counter (the
message_count_send sums of node.py:114-116) and every seen bit must equal a run that reads them
each round (P2PG_RUN_BATCH=1, step by step), and the C oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ("new_deliveries", "relays", "active_vertices", "active_words", "wedges", "deg_active",
          "scatter_words", "touched_words")


def _net(g, thr, **kw):
    from p2pnetwork.gpu import GraphNetwork
    return GraphNetwork(g, mode="gossip", fanout=3, gossip_seed=0x5EED, churn_threshold_value=thr,
                        churn_seed=0xC0FFEE, **kw)


def _log(msg):
    import sys
    import time
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)
    sys.stdout.flush()


def _rows(rounds):
    return [tuple(getattr(r, f) for f in FIELDS) for r in rounds]


# BA m=4 (config 4's graph) with and without churn; WS k=8 with churn, whose decay tail is not
# monotone (lost sends leave pockets that later rounds still reach), so the batched tail's list
# bound is exercised on a tail it does not shrink evenly
@pytest.mark.parametrize("kind,thr", [("ba", 0), ("ba", 200_000_000), ("ws", 400_000_000)])
def test_batched_and_blind_rounds_equal_round_by_round(kind, thr, monkeypatch):
    from oracle import coracle
    from p2pnetwork.gpu import PeerGraph, make_sources
    g = (PeerGraph.barabasi_albert(1_000_000, 4, seed=5) if kind == "ba"
         else PeerGraph.watts_strogatz(300_000, 8, 0.1, seed=5))
    src = make_sources(g.V, 4096, seed=3)
    with _net(g, thr) as net:                         # p2pg_run: batched decay tail
        net.broadcast(src)
        a = net.run()
        _log(f"batched run: {len(a)} rounds")
        seen_a = net.seen_plane()
        assert len(net.deliveries(cap=16)) == 0       # quiescent: no receipts in the last round
        net.reset()
        chunked = []
        while True:                                   # p2pg_run in chunks of 3 rounds
            part = net.run(max_rounds=3)
            chunked += part
            if not part[-1].active:
                break
        seen_c = net.seen_plane()
        _log(f"chunked run: {len(chunked)} rounds")
    monkeypatch.setenv("P2PG_RUN_BATCH", "1")
    with _net(g, thr) as net:                         # p2pg_run, one synchronisation per round
        net.broadcast(src)
        b = net.run()
        _log(f"unbatched run: {len(b)} rounds")
        seen_b = net.seen_plane()
    with _net(g, thr) as net:                         # p2pg_step, one round per call
        net.broadcast(src)
        c = []
        while True:
            st = net.step()
            c.append(st)
            if not st.active:
                break
        seen_s = net.seen_plane()
        _log(f"step run: {len(c)} rounds")
    assert _rows(a) == _rows(b) == _rows(c) == _rows(chunked)
    for s in (seen_b, seen_c, seen_s):
        np.testing.assert_array_equal(seen_a, s)
    _log("oracle")
    ora = coracle.run(g.rowptr, g.colidx, src, "gossip", 3, 0x5EED, 0, thr, 0xC0FFEE, record=False,
                      want_seen=True)
    np.testing.assert_array_equal(seen_a, ora.seen)
    want = [tuple(r[f] for f in FIELDS[:-1]) for r in ora.rounds]
    assert [x[:-1] for x in _rows(a)][:len(want)] == want


def test_new_sources_and_resets_recount_round_zero():
    """Round 0's counters come from the host copy of the sources (cached per sources and graph,
    engine.cpp seed_stats): a second broadcast() with other sources on the same engine, and a
    reset between runs (the double-buffered seen plane swaps in its zeroed spare), give exactly a
    fresh engine's rounds -- counters and seen plane -- each time."""
    from p2pnetwork.gpu import PeerGraph, make_sources
    g = PeerGraph.barabasi_albert(300_000, 4, seed=11)
    a, b = make_sources(g.V, 4096, seed=1), make_sources(g.V, 1000, seed=2)
    ref = {}
    for name, src in (("a", a), ("b", b)):
        with _net(g, 0) as net:
            net.broadcast(src)
            ref[name] = (_rows(net.run()), net.seen_plane())
    with _net(g, 0) as net:
        for name, src in (("a", a), ("b", b), ("a", a)):
            net.broadcast(src)
            for _ in range(2):
                net.reset()
                rows = _rows(net.run())
                assert rows == ref[name][0], name
                np.testing.assert_array_equal(net.seen_plane(), ref[name][1], err_msg=name)


@pytest.mark.parametrize("M", [1536, 2560, 4096])  # W = 24 / 40 / 64: packed rows (AW planes)
def test_partial_frontier_rows_every_push_form(M, monkeypatch):
    """Inside p2pg_run, updates and the last dense pull write only the nonzero words of their
    frontier rows (store_f == 2: the rows are valid under their AW masks only).  Every reader of
    those rows -- the sparse push list, the per-source scatter, the fused push-only pass -- must
    read them through AW: whole-row writes (P2PG_PARTIAL_F=0) give identical rounds and seen
    planes, in each push form (default, unfused per-source scatter, per-source sparse push)."""
    from p2pnetwork.gpu import PeerGraph, make_sources
    g = PeerGraph.barabasi_albert(400_000, 4, seed=12)
    src = make_sources(g.V, M, seed=13)
    forms = {"auto": {}, "no_push_fused": {"P2PG_PUSH_FUSED": "0"},
             "per_source_sparse": {"P2PG_SPARSE_LP": "0"}}
    ref = None
    for name, env in forms.items():
        for partial in ("1", "0"):
            for k in ("P2PG_PUSH_FUSED", "P2PG_SPARSE_LP"):
                monkeypatch.delenv(k, raising=False)
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            monkeypatch.setenv("P2PG_PARTIAL_F", partial)
            with _net(g, 0) as net:
                net.broadcast(src)
                rows = _rows(net.run())
                seen = net.seen_plane()
            if ref is None:
                ref = (rows, seen)
                continue
            assert [r[:-1] for r in rows] == [r[:-1] for r in ref[0]], (name, partial)
            np.testing.assert_array_equal(seen, ref[1], err_msg=f"{name} partial={partial}")
