"""GPU parity of the vertex-partitioned path: every rank is a real HIP engine (C-ABI
partition entry points: global ids, exchange lists, pack/unpack kernels) on cuda:0, the ranks
run as threads of one process and a thread transport stands in for the all-to-all.  The union
of the owned results must equal the single-engine run and the oracle bit for bit."""
import threading
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import trim_zeros
from oracle import coracle, relay_oracle

pytestmark = pytest.mark.gpu


class ThreadTransport:
    """The transport contract of PartitionedNetwork among `world` threads of one process
    (device tensors): an all-gather of count vectors and the record sends / receives."""

    def __init__(self, shared, rank):
        self.s, self.rank = shared, rank
        self.rows_total = self.rows_sent = 0

    def _gather(self, item):
        s = self.s
        s["slots"][self.rank] = item
        s["barrier"].wait()
        items = list(s["slots"])
        s["barrier"].wait()
        return items

    def engine_stream(self):
        # as TorchTransport on a GPU: the engine gets a torch stream, and the unpack waits for
        # the copies below by a stream wait (PartitionedNetwork._ready), not a host sync
        import torch
        return torch.cuda.Stream(device=0)

    def exchange_counts(self, vec):
        return np.stack(self._gather(np.asarray(vec, dtype=np.int64)))

    def exchange_records(self, send_buf, send_off, send_cnt, recv_buf, recv_cnt, R):
        # no extra synchronisation: the production ordering (PartitionedNetwork._ready) is tested
        items = self._gather((send_buf, np.asarray(send_off), np.asarray(send_cnt)))
        off = 0
        for p, (buf, so, sc) in enumerate(items):
            n = int(sc[self.rank]) if p != self.rank else 0
            assert n == int(recv_cnt[p]) or p == self.rank
            if n:
                recv_buf[off * R:(off + n) * R].copy_(buf[int(so[self.rank]) * R:(int(so[self.rank]) + n) * R])
                off += n
        self.s["barrier"].wait()  # every rank has copied out of the send buffers


def run_partitioned(g, world, src, overlap=True, forms=None, **kw):
    """forms: a list that receives each rank's local push forms (round stats' push_form)."""
    from p2pnetwork.gpu import PartitionedNetwork
    shared = {"slots": [None] * world, "barrier": threading.Barrier(world)}
    results, errors = [None] * world, []
    if forms is not None:
        forms[:] = [None] * world

    def rank_main(rank):
        try:
            net = PartitionedNetwork(g, world, rank, ThreadTransport(shared, rank), overlap=overlap, **kw)
            with net.net:
                net.broadcast(src)
                rounds = net.run()
                gids, seen = net.owned_planes()
                hp = net.owned_hop_parent() if kw.get("record") else None
            results[rank] = (rounds, gids, seen, hp)
            if forms is not None:
                forms[rank] = [r.push_form for r in net.local_rounds]
        except BaseException as exc:  # surface in the main thread; unblock the others
            errors.append(exc)
            shared["barrier"].abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    if errors:
        raise errors[0]
    return results


def assemble(results, V, W):
    seen = np.zeros((V, W), dtype=np.uint64)
    for _, gids, s, _ in results:
        seen[gids] = s
    return seen


def graph(kind):
    from p2pnetwork.gpu import PeerGraph
    if kind == "ws":
        return PeerGraph.watts_strogatz(20_000, 8, 0.1, seed=3)
    if kind == "ba":
        return PeerGraph.barabasi_albert(30_000, 4, seed=7)   # hubs at low ids -> hub kernels
    return PeerGraph.gnp(5_000, 1.5, seed=2)                   # many small components


@pytest.mark.parametrize("kind,mode,M,thr,world,overlap", [
    ("ws", "flood", 64, 0, 2, True),
    ("ws", "flood", 64, 0, 2, False),
    ("ws", "flood", 130, 400_000_000, 3, True),
    ("ba", "flood", 200, 0, 4, True),
    ("sparse", "flood", 65, 0, 3, True),
    ("ws", "gossip", 64, 0, 2, True),
    ("ws", "gossip", 64, 0, 2, False),
    ("ba", "gossip", 96, 300_000_000, 3, True),
    ("sparse", "gossip", 40, 0, 4, True),
])
def test_partitioned_engines_match_single_gpu(kind, mode, M, thr, world, overlap):
    """Real engines as threads == one engine == the C oracle; compacted record exchange (only
    boundary rows with a non-zero word travel), with the next round's interior peers running
    while the records are exchanged (overlap) and without."""
    from p2pnetwork.gpu import GraphNetwork, make_sources
    g = graph(kind)
    src = make_sources(g.V, M, seed=21)
    kw = dict(mode=mode, fanout=3, gossip_seed=99, churn_threshold_value=thr, churn_seed=17)
    res = run_partitioned(g, world, src, overlap=overlap, record=True, **kw)
    with GraphNetwork(g, record=True, **kw) as one:
        one.broadcast(src)
        rounds1 = one.run()
        seen1 = one.seen_plane()
        hop1, par1 = one.hop_parent()
    W = (M + 63) // 64
    np.testing.assert_array_equal(assemble(res, g.V, W), seen1)
    keys = ("new_deliveries", "relays", "active_vertices", "active_words", "wedges", "deg_active",
            "scatter_words")
    for rounds, *_ in res:  # every rank reports the global counters
        for k in keys:
            np.testing.assert_array_equal(trim_zeros([getattr(r, k) for r in rounds]),
                                          trim_zeros([getattr(r, k) for r in rounds1]), err_msg=k)
    # hop / parent of every owned peer (gossip: ghost senders' picks replayed from their global
    # degree and adjacency order, their frontier rows exchanged as plane 0)
    hop = np.full((g.V, M), -1, np.int32)
    par = np.full((g.V, M), -1, np.int32)
    for _, _, _, (gids, h, p) in res:
        hop[gids], par[gids] = h, p
    np.testing.assert_array_equal(hop, hop1)
    np.testing.assert_array_equal(par, par1)
    # and the single engine against the oracle (C restatement)
    ora = coracle.run(g.rowptr, g.colidx, src, mode, 3, 99, 0, thr, 17, record=True)
    np.testing.assert_array_equal(hop1, ora.hop)
    np.testing.assert_array_equal(par1, ora.parent)


# Every origin inside the LAST rank's id block (Watts-Strogatz: the other ranks are reached late,
# only through exchanged rows): a rank's own pushed-mask count then says nothing about the frontier
# the exchange hands it, so a partitioned rank never pushes blind and sizes its (peer, word) list
# by its own counters (advisor, round 4).  Narrow rows (row atomics only on partitioned ranks) and
# the packed dense form, with churn.
@pytest.mark.parametrize("M,world,thr", [(1024, 2, 0), (4096, 3, 300_000_000)])
def test_partitioned_gossip_sources_in_one_block(M, world, thr):
    from p2pnetwork.gpu import GraphNetwork, VertexPartition
    g = graph("ws")
    bounds = VertexPartition.ranges(g, world)
    lo, hi = int(bounds[world - 1]), int(bounds[world])
    rng = np.random.default_rng(5)
    src = rng.integers(lo, hi, size=M).astype(np.int32)
    kw = dict(mode="gossip", fanout=3, gossip_seed=31, churn_threshold_value=thr, churn_seed=8)
    res = run_partitioned(g, world, src, **kw)
    with GraphNetwork(g, **kw) as one:
        one.broadcast(src)
        rounds1 = one.run()
        seen1 = one.seen_plane()
    np.testing.assert_array_equal(assemble(res, g.V, (M + 63) // 64), seen1)
    for rounds, *_ in res:
        for k in ("new_deliveries", "relays", "active_vertices", "active_words"):
            np.testing.assert_array_equal(trim_zeros([getattr(r, k) for r in rounds]),
                                          trim_zeros([getattr(r, k) for r in rounds1]), err_msg=k)


# Partitioned ranks take gossip's dense rounds at 16 < W <= 64 (relay_kernels.hip PART kernels):
# E planes for local connections, row pushes for ghost connections (exchanged as plane 1) ORed
# into the gather of the next round.  Widths 24 / 32 (two slots per gather load) / 64, the engine's
# own schedule and every round forced dense (P2PG_GOSSIP_PUSH=store), churn, hubs on one rank,
# records (hop / parent, ghost senders): == one engine == the C oracle.
@pytest.mark.parametrize("kind,M,world,thr,env", [
    ("ba", 1536, 3, 300_000_000, {"P2PG_GOSSIP_PUSH": "store"}),
    ("ba", 2048, 2, 0, {"P2PG_V_THRESH": "0.2"}),
    ("ws", 4096, 4, 200_000_000, {"P2PG_V_THRESH": "0.2"}),
    ("ws", 1100, 3, 0, {"P2PG_GOSSIP_PUSH": "store"}),
])
def test_partitioned_gossip_dense_rounds(kind, M, world, thr, env, monkeypatch):
    from p2pnetwork.gpu import GraphNetwork, make_sources
    from p2pnetwork.gpu.network import PUSH_FORMS
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = graph(kind)
    src = make_sources(g.V, M, seed=31)
    kw = dict(mode="gossip", fanout=3, gossip_seed=77, churn_threshold_value=thr, churn_seed=23)
    forms = []
    res = run_partitioned(g, world, src, overlap=True, forms=forms, record=True, **kw)
    dense = {PUSH_FORMS.index("edge"), PUSH_FORMS.index("fused")}
    assert all(any(f in dense for f in fr) for fr in forms), forms
    assert any(PUSH_FORMS.index("fused") in fr for fr in forms), forms
    with GraphNetwork(g, record=True, **kw) as one:
        one.broadcast(src)
        rounds1 = one.run()
        seen1 = one.seen_plane()
        hop1, par1 = one.hop_parent()
    np.testing.assert_array_equal(assemble(res, g.V, (M + 63) // 64), seen1)
    for rounds, *_ in res:
        _assert_same_rounds(rounds, rounds1)
    hop = np.full((g.V, M), -1, np.int32)
    par = np.full((g.V, M), -1, np.int32)
    for _, _, _, (gids, h, p) in res:
        hop[gids], par[gids] = h, p
    np.testing.assert_array_equal(hop, hop1)
    np.testing.assert_array_equal(par, par1)
    ora = coracle.run(g.rowptr, g.colidx, src, "gossip", 3, 77, 0, thr, 23, record=True)
    np.testing.assert_array_equal(hop1, ora.hop)
    np.testing.assert_array_equal(par1, ora.parent)


@pytest.mark.parametrize("kind,mode,world", [("ba", "gossip", 3), ("ws", "flood", 4), ("sparse", "gossip", 2)])
def test_partitioned_delivery_stream(kind, mode, world):
    """The batched node_message hook on a vertex partition: per round, the union over ranks of
    each rank's owned first receipts (global peer ids, parent = the sender of node.py:334-338)
    == the single engine's delivery stream, record for record."""
    from p2pnetwork.gpu import GraphNetwork, PartitionedNetwork, make_sources
    g = graph(kind)
    src = make_sources(g.V, 70, seed=4)
    kw = dict(mode=mode, fanout=3, gossip_seed=5, churn_threshold_value=200_000_000, churn_seed=9)
    shared = {"slots": [None] * world, "barrier": threading.Barrier(world)}
    per_rank, errors = [None] * world, []

    def rank_main(rank):
        try:
            net = PartitionedNetwork(g, world, rank, ThreadTransport(shared, rank), deliveries=True, **kw)
            out = []
            with net.net:
                net.broadcast(src)
                while True:
                    st = net.step()
                    out.append(net.deliveries())
                    if not st.new_deliveries:
                        break
            per_rank[rank] = out
        except BaseException as exc:
            errors.append(exc)
            shared["barrier"].abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    if errors:
        raise errors[0]
    with GraphNetwork(g, **kw) as one:
        one.broadcast(src)
        want = []
        while True:
            st = one.step()
            want.append(one.deliveries())
            if not st.active:
                break
    n = max(len(want), *(len(x) for x in per_rank))
    for r in range(n):
        got = [x[r] for x in per_rank if r < len(x)]
        peer = np.concatenate([d.peer for d in got])
        order = np.lexsort((np.concatenate([d.msg for d in got]), peer))
        w = want[r] if r < len(want) else None
        if w is None:
            assert len(peer) == 0
            continue
        for f in ("peer", "msg", "hop", "parent"):
            np.testing.assert_array_equal(np.concatenate([getattr(d, f) for d in got])[order],
                                          getattr(w, f), err_msg=f"round {r} {f}")


def test_partitioned_gossip_small_matches_numpy_oracle():
    from p2pnetwork.gpu import PeerGraph, make_sources
    g = PeerGraph.watts_strogatz(300, 6, 0.3, seed=1)
    src = make_sources(g.V, 33, seed=2)
    res = run_partitioned(g, 3, src, mode="gossip", fanout=2, gossip_seed=5,
                          churn_threshold_value=900_000_000, churn_seed=8)
    ora = relay_oracle.gossip(g.rowptr, g.colidx, src, 2, 5, 0, 900_000_000, 8)
    seen = assemble(res, g.V, 1)
    bits = np.unpackbits(seen.view(np.uint8), axis=1, bitorder="little")[:, :33].astype(bool)
    np.testing.assert_array_equal(bits, ora.hop >= 0)
    np.testing.assert_array_equal(trim_zeros([r.relays for r in res[0][0]]),
                                  trim_zeros([r["relays"] for r in ora.rounds]))


# --- the multi-GPU forms at their real widths (W = 64, 8 ranks), on the one GPU ---------------
# config 5's job (bench.py --workload c5 --gpus 8) packs records of 1 + 64 int64 per live row
# across 8 list segments with the next round's interior peers overlapping the exchange; here that
# combination runs with real engines (8 thread-ranks on cuda:0) at 1M peers before any 8-GPU job
# does, against one engine and against the C oracle (nodeconnection.py:107-160 is the fan-out it
# replaces, node.py:106-120 the relay).

def _c5_like():
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.network import churn_threshold
    return PeerGraph.watts_strogatz(1_000_000, 8, 0.1, seed=5), churn_threshold(0.05)


def _round_keys(rounds):
    keys = ("new_deliveries", "relays", "active_vertices", "active_words", "wedges", "deg_active",
            "scatter_words")
    return {k: trim_zeros([getattr(r, k) for r in rounds]) for k in keys}


def _assert_same_rounds(got, want):
    a, b = _round_keys(got), _round_keys(want)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_partitioned_8_ranks_full_width_flood_churn():
    """8 ranks, WS k=8 beta=0.1 at 1M peers, 4096 floods (W = 64), churn 0.05, overlap on: the
    assembled seen plane and every global per-round counter == one engine; words 0 and 63 ==
    64-broadcast partitioned runs whose hop / parent planes == the C oracle's bit for bit."""
    from p2pnetwork.gpu import GraphNetwork, make_sources
    g, thr = _c5_like()
    M, world = 4096, 8
    src = make_sources(g.V, M, seed=1)
    kw = dict(mode="flood", churn_threshold_value=thr, churn_seed=0xC0FFEE)
    res = run_partitioned(g, world, src, overlap=True, **kw)
    with GraphNetwork(g, **kw) as one:
        one.broadcast(src)
        rounds1 = one.run()
        seen1 = one.seen_plane()
    seen = assemble(res, g.V, M // 64)
    np.testing.assert_array_equal(seen, seen1)
    for rounds, *_ in res:
        _assert_same_rounds(rounds, rounds1)
    for w in (0, 63):
        s = src[64 * w:64 * (w + 1)]
        part = run_partitioned(g, world, s, overlap=True, record=True, **kw)
        np.testing.assert_array_equal(assemble(part, g.V, 1)[:, 0], seen[:, w], err_msg=f"word {w}")
        hop = np.full((g.V, 64), -1, np.int32)
        par = np.full((g.V, 64), -1, np.int32)
        for _, _, _, (gids, h, p) in part:
            hop[gids], par[gids] = h, p
        ora = coracle.run(g.rowptr, g.colidx, s, "flood", 3, 0, 0, thr, 0xC0FFEE, record=True)
        np.testing.assert_array_equal(hop, ora.hop, err_msg=f"word {w} hop")
        np.testing.assert_array_equal(par, ora.parent, err_msg=f"word {w} parent")
        _assert_same_rounds(part[0][0], [SimpleNamespace(**r) for r in ora.rounds])


def test_partitioned_8_ranks_full_width_gossip():
    """Gossip (k = 3, churn 0.05) over 8 ranks at W = 64 on a 1M-peer BA graph (hubs at the low
    ids, on rank 0; every rank runs fused dense rounds): the assembled seen plane and the global per-round counters == one engine;
    words 0 and 63 == the C oracle's delivered sets (their broadcasts run alone, with their global
    message ids)."""
    from p2pnetwork.gpu import GraphNetwork, PeerGraph, make_sources
    from p2pnetwork.gpu.network import churn_threshold
    g = PeerGraph.barabasi_albert(1_000_000, 4, seed=11)
    thr = churn_threshold(0.05)
    M, world = 4096, 8
    src = make_sources(g.V, M, seed=1)
    kw = dict(mode="gossip", fanout=3, gossip_seed=0x5EED, churn_threshold_value=thr, churn_seed=0xC0FFEE)
    forms = []
    res = run_partitioned(g, world, src, overlap=True, forms=forms, **kw)
    # the dense rounds run on the ranks too (PART kernels), not row atomics only
    from p2pnetwork.gpu.network import PUSH_FORMS
    assert all(PUSH_FORMS.index("fused") in fr for fr in forms), forms
    with GraphNetwork(g, **kw) as one:
        one.broadcast(src)
        rounds1 = one.run()
        seen1 = one.seen_plane()
    seen = assemble(res, g.V, M // 64)
    np.testing.assert_array_equal(seen, seen1)
    for rounds, *_ in res:
        _assert_same_rounds(rounds, rounds1)
    for w in (0, 63):
        ora = coracle.run(g.rowptr, g.colidx, src[64 * w:64 * (w + 1)], "gossip", 3, 0x5EED, 64 * w, thr,
                          0xC0FFEE, record=False, want_seen=True)
        np.testing.assert_array_equal(seen[:, w], ora.seen[:, 0], err_msg=f"word {w}")
