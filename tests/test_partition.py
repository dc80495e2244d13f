"""Vertex-partitioned multi-GPU path (p2pnetwork.gpu.partition), exercised on CPU with the
gloo backend (world sizes 2, 3 and 8) through the real orchestration code; each rank's engine is
the test-only NumPy stand-in of tests/partition_mock.py.  The union of the ranks' owned
results must equal the single-graph oracle bit for bit (hop, parent, per-round counters)."""
import os
import socket
import tempfile

import numpy as np
import pytest

from conftest import trim_zeros
from oracle import relay_oracle


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_graph(kind):
    from p2pnetwork.gpu import PeerGraph
    if kind == "ws":
        return PeerGraph.watts_strogatz(240, 6, 0.2, seed=4)
    if kind == "ba":
        return PeerGraph.barabasi_albert(200, 3, seed=5)
    edges = [(0, 1), (1, 2), (5, 6), (8, 9)]  # sparse: isolated peers, tiny components
    return PeerGraph.from_edges(30, edges)


@pytest.mark.parametrize("world", [1, 2, 3, 4])
@pytest.mark.parametrize("kind", ["ws", "ba", "sparse"])
def test_partition_lists_are_symmetric_and_cover(world, kind):
    from p2pnetwork.gpu import VertexPartition
    g = make_graph(kind)
    parts = [VertexPartition(g, world, r) for r in range(world)]
    owned = np.concatenate([p.gid[p.owned_local] for p in parts])
    assert np.array_equal(np.sort(owned), np.arange(g.V))
    for q in range(world):
        pq = parts[q]
        so = np.concatenate([[0], np.cumsum(pq.send_counts)])
        for p in range(world):
            pp = parts[p]
            ro = np.concatenate([[0], np.cumsum(pp.recv_counts)])
            sent = pq.gid[pq.send_local[so[p]:so[p + 1]]]
            got = pp.gid[pp.recv_local[ro[q]:ro[q + 1]]]
            assert np.array_equal(sent, got)
        lg = pq.local_graph()
        lg.rowptr.shape  # local rows: owned rows hold every global neighbour, ascending
        for u in pq.owned_local[:20]:
            nb_local = lg.colidx[lg.rowptr[u]:lg.rowptr[u + 1]]
            assert np.array_equal(pq.gid[nb_local], g.neighbours(pq.gid[u]))


def _rank_main(rank, world, port, kind, mode, M, thr, out, overlap=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "python-p2p-network_amd"), here):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from p2pnetwork.gpu import PartitionedNetwork, TorchTransport, make_sources
    from partition_mock import MockEngine
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = make_graph(kind)
    src = make_sources(g.V, M, seed=11)
    tr = TorchTransport()
    net = PartitionedNetwork(g, world, rank, tr, mode=mode, fanout=3,
                             gossip_seed=77, churn_threshold_value=thr, churn_seed=5,
                             engine_factory=MockEngine, overlap=overlap)
    net.broadcast(src)
    rounds = net.run()
    gids, seen = net.owned_planes()
    _, hop, par = net.owned_hop_parent()
    np.savez(os.path.join(out, f"rank{rank}.npz"), gids=gids, hop=hop, par=par,
             relays=np.array([r.relays for r in rounds]), new=np.array([r.new_deliveries for r in rounds]),
             words=np.array([r.active_words for r in rounds]), scatter=np.array([r.scatter_words for r in rounds]),
             rows=np.array([tr.rows_sent, tr.rows_total]))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,mode,M,thr,world,overlap", [
    ("ws", "flood", 70, 0, 2, True),
    ("ws", "flood", 70, 0, 2, False),
    ("ws", "flood", 64, 600_000_000, 3, True),
    ("sparse", "flood", 40, 0, 2, True),
    ("ba", "gossip", 64, 0, 2, True),
    ("ba", "gossip", 64, 0, 2, False),
    ("ws", "gossip", 30, 500_000_000, 3, True),
    # the 8 ranks config 5 runs on one node
    ("ws", "flood", 70, 300_000_000, 8, True),
    ("ba", "gossip", 64, 0, 8, True),
    ("ws", "gossip", 96, 200_000_000, 8, False),
])
def test_partitioned_gloo_matches_oracle(kind, mode, M, thr, world, overlap):
    """Ranks over gloo (stand-in engines) == the oracle, with the compacted record exchange
    (only boundary rows with a non-zero word travel: one all-gather of counts, grouped
    sends / receives), with and without the next round begun during the exchange."""
    import torch.multiprocessing as mp
    from p2pnetwork.gpu import make_sources
    g = make_graph(kind)
    src = make_sources(g.V, M, seed=11)
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_rank_main, args=(world, free_port(), kind, mode, M, thr, out, overlap), nprocs=world,
                           start_method="spawn")
        parts = [dict(np.load(os.path.join(out, f"rank{r}.npz"))) for r in range(world)]
    hop = np.full((g.V, M), -1, np.int32)
    par = np.full((g.V, M), -1, np.int32)
    for p in parts:
        hop[p["gids"]] = p["hop"]
        par[p["gids"]] = p["par"]
    if mode == "flood":
        ora = relay_oracle.flood(g.rowptr, g.colidx, src, thr, 5)
        np.testing.assert_array_equal(par, ora.parent)
    else:
        ora = relay_oracle.gossip(g.rowptr, g.colidx, src, 3, 77, 0, thr, 5)
    np.testing.assert_array_equal(hop, ora.hop)
    r0 = parts[0]
    sent, offered = sum(p["rows"][0] for p in parts), sum(p["rows"][1] for p in parts)
    assert sent < offered or offered == 0  # dead boundary rows stayed home
    for p in parts[1:]:  # every rank reports the same global counters
        for k in ("relays", "new", "words", "scatter"):
            np.testing.assert_array_equal(p[k], r0[k])
    np.testing.assert_array_equal(trim_zeros(r0["relays"]), trim_zeros([r["relays"] for r in ora.rounds]))
    np.testing.assert_array_equal(trim_zeros(r0["new"]), trim_zeros([r["new_deliveries"] for r in ora.rounds]))
    np.testing.assert_array_equal(trim_zeros(r0["words"]), trim_zeros([r["active_words"] for r in ora.rounds]))
    np.testing.assert_array_equal(trim_zeros(r0["scatter"]), trim_zeros([r["scatter_words"] for r in ora.rounds]))


def test_partition_refuses_more_ranks_than_the_exchange_holds():
    from p2pnetwork.gpu import PartitionedNetwork
    from partition_mock import MockEngine
    g = make_graph("ws")
    with pytest.raises(ValueError, match="1..16"):
        PartitionedNetwork(g, 17, 0, transport=None, engine_factory=MockEngine)


@pytest.mark.parametrize("world", [2, 3, 5])
def test_ghost_senders_positions(world):
    """VertexPartition.ghost_senders: for every local slot whose neighbour u is a ghost, the
    row owner's position in u's GLOBAL ascending adjacency and u's global degree (what replaying
    a remote gossip sender's Floyd picks needs, node.py:114-120); -1 for local neighbours."""
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.partition import VertexPartition
    g = PeerGraph.barabasi_albert(2000, 3, seed=world)
    for r in range(world):
        P = VertexPartition(g, world, r)
        gdeg, pos = P.ghost_senders(g)
        nb = P.gid[P.colidx].astype(np.int64)
        owner = P.gid[np.searchsorted(P.rowptr, np.arange(len(P.colidx)), side="right") - 1]
        remote = (nb < P.lo) | (nb >= P.hi)
        assert np.array_equal(pos >= 0, remote)
        for j in np.nonzero(remote)[0]:
            row = g.colidx[g.rowptr[nb[j]]:g.rowptr[nb[j] + 1]]
            assert row[pos[j]] == owner[j]
            assert gdeg[P.colidx[j]] == len(row)
