"""RCCL on the one-GPU box (child process of tests/test_gpu_rccl.py, started before anything in it
touches the GPU): the RCCL-specific pieces of a vertex-partitioned job, which otherwise first run
in the driver's 8-GPU bench.

1. ``init_process_group("nccl", device_id=cuda:0)`` at world 1, ``host_group_for`` (a gloo
   group next to the nccl one) and ``TorchTransport`` over them, whose count all-gather goes
   over gloo;
2. two ranks of a vertex partition, as threads of this process, each with a transport that IS
   ``TorchTransport`` -- its own ``exchange_records`` (compaction per destination, split sizes,
   gloo staging rules, stream order) -- except for the one collective primitive
   ``_all_to_all``: RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so the two
   logical ranks' all-to-alls are issued as ONE world-1 RCCL ``all_to_all_single`` with split
   sizes (the call of production, at world 1 a device copy) over both ranks' chunks, and the
   engines order ``p2pg_exchange_unpack_live`` after it with ``PartitionedNetwork._ready``'s
   ``wait_stream``;
3. the partitioned runs (flood with churn, gossip with churn, W = 64) == one engine, bit for bit.

Replaces, like the rest of the partition layer, the cross-host fan-out of NodeConnection.send
(p2pnetwork/nodeconnection.py:107-160).  Prints one line starting with "RCCL OK" on success."""
import os
import sys
import threading

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "python-p2p-network_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from p2pnetwork.gpu import TorchTransport  # noqa: E402


class RcclLoopback(TorchTransport):
    """Logical rank `rank` of `world` rank threads of one process over the world-1 RCCL group:
    TorchTransport with the collective primitive (and the count all-gather) met in a shared slot
    table; rank 0's thread issues the one RCCL all_to_all_single per round."""

    def __init__(self, shared, rank, world, tt):
        super().__init__(device=tt.device, host_group=tt.host_group)
        self.world, self.rank = world, rank  # logical
        self.s, self.tt = shared, tt

    def _gather(self, item):
        s = self.s
        s["slots"][self.rank] = item
        s["barrier"].wait()
        items = list(s["slots"])
        s["barrier"].wait()
        return items

    def exchange_counts(self, vec):
        allv = np.stack(self._gather(np.asarray(vec, dtype=np.int64)))
        if self.rank == 0:  # the gloo group next to the nccl communicator, every round
            got = self.tt.exchange_counts(allv.reshape(-1))
            assert np.array_equal(got.reshape(-1), allv.reshape(-1)), "gloo all-gather"
        return allv

    def _all_to_all(self, out, inp, out_splits, in_splits):
        items = self._gather((out, inp, list(out_splits), list(in_splits)))
        if self.rank == 0:
            W = len(items)
            # destination q's chunk from source p: p's input at offset sum(in_splits[:q]);
            # q's output takes its sources in order -- one input / output pair in (q, p) order
            ins, outs = [], []
            for q in range(W):
                for p in range(W):
                    n = items[p][3][q]
                    assert n == items[q][2][p], "split sizes disagree"
                    if n:
                        a = sum(items[p][3][:q])
                        ins.append(items[p][1][a:a + n])
                        b = sum(items[q][2][:p])
                        outs.append(items[q][0][b:b + n])
            total = sum(x.numel() for x in ins)
            if total:
                x = torch.cat(ins)
                y = torch.empty_like(x)
                dist.all_to_all_single(y, x, [total], [total])  # RCCL kernel, current stream
                o = 0
                for t in outs:
                    t.copy_(y[o:o + t.numel()])
                    o += t.numel()
            self.s["moved"] += total
            self.s["calls"] += 1
        self.s["barrier"].wait()  # the copies are enqueued before any rank unpacks


def run_case(tt, g, src, world, **kw):
    from p2pnetwork.gpu import GraphNetwork, PartitionedNetwork
    shared = {"slots": [None] * world, "barrier": threading.Barrier(world), "moved": 0, "calls": 0}
    res, errors = [None] * world, []

    def rank_main(rank):
        try:
            torch.cuda.set_device(0)
            net = PartitionedNetwork(g, world, rank, RcclLoopback(shared, rank, world, tt), **kw)
            with net.net:
                net.broadcast(src)
                rounds = net.run()
                res[rank] = (rounds, *net.owned_planes())
        except BaseException as exc:
            errors.append(exc)
            shared["barrier"].abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    if errors:
        raise errors[0]
    with GraphNetwork(g, **kw) as one:
        one.broadcast(src)
        rounds1 = one.run()
        seen1 = one.seen_plane()
    seen = np.zeros_like(seen1)
    for _, gids, s in res:
        seen[gids] = s
    assert np.array_equal(seen, seen1), "partitioned seen plane != one engine"
    keys = ("new_deliveries", "relays", "active_vertices", "active_words", "wedges", "deg_active",
            "scatter_words")
    for rounds, *_ in res:
        for k in keys:
            a = [getattr(r, k) for r in rounds]
            b = [getattr(r, k) for r in rounds1]
            while a and a[-1] == 0:
                a.pop()
            while b and b[-1] == 0:
                b.pop()
            assert a == b, k
    assert shared["moved"] > 0, "no record moved through RCCL"
    # one all-to-all per exchange (frontier rows per round; gossip also its senders' rows)
    assert shared["calls"] >= len(rounds1) - 1
    return len(rounds1), shared["moved"] // (1 + len(src) // 64)


def main():
    assert os.environ.get("WORLD_SIZE") == "1" and os.environ.get("MASTER_ADDR") == "127.0.0.1"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    from p2pnetwork.gpu import PeerGraph, TorchTransport, make_sources
    from p2pnetwork.gpu.network import churn_threshold
    from p2pnetwork.gpu.partition import host_group_for
    hg = host_group_for(None)
    tt = TorchTransport(device=torch.device("cuda", 0), host_group=hg)
    assert tt.backend == "nccl" and tt.world == 1
    assert np.array_equal(tt.exchange_counts(np.array([3, 5, 7])), [[3, 5, 7]])
    # one RCCL collective on device tensors by itself first, and TorchTransport's own exchange
    # at world 1 (no other rank: an empty all-to-all, as a rank with nothing to send makes it)
    x = torch.arange(1 << 20, dtype=torch.int64, device="cuda:0")
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x)
    assert torch.equal(x, y)
    tt.exchange_records(x, np.array([0]), np.array([0]), y, np.array([0]), 65)
    assert tt.collectives == 1
    thr = churn_threshold(0.05)
    out = []
    g = PeerGraph.watts_strogatz(40_000, 8, 0.1, seed=9)
    out.append(("flood", *run_case(tt, g, make_sources(g.V, 4096, seed=3), 2, mode="flood",
                                   churn_threshold_value=thr, churn_seed=0xC0FFEE)))
    g = PeerGraph.barabasi_albert(40_000, 4, seed=9)
    out.append(("gossip", *run_case(tt, g, make_sources(g.V, 4096, seed=3), 2, mode="gossip", fanout=3,
                                    gossip_seed=0x5EED, churn_threshold_value=thr, churn_seed=0xC0FFEE)))
    dist.destroy_process_group()
    print("RCCL OK " + " ".join(f"{m}: {n} rounds, {r} records through RCCL;" for m, n, r in out), flush=True)


if __name__ == "__main__":
    main()
