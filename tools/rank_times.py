"""Per-rank kernel time of a multi-GPU form of config 4, each rank ALONE on the one GPU
(development aid for DESIGN.md section 6's table of N-GPU forms).

    python tools/rank_times.py <vertex ranks> <broadcasts> [steps] > gpurun_out/ranks_<N>.json

The ranks of a vertex partition (PartitionedNetwork engines, W = ceil(broadcasts / 64)) are
driven round by round from ONE thread: rank 0's round, then rank 1's, ... each finished (stream
synchronised) before the next starts, so no two ranks share the GPU; then the live records move
between the ranks' buffers by device copies and are unpacked.  Per round and rank it records the
engine's kernel time (HIP events) and the record bytes sent / received, and projects an N-GPU
step as sum over rounds of (slowest rank's kernels + the round's exchange at XGMI_GBPS per
direction, not overlapped).  "broadcasts" < 4096 is one group of a message x vertex form: the
group's ranks run messages [0, broadcasts) with their global ids; the other groups' shares are
the same work on other messages.  The global per-round counters are checked against one engine
run of the same broadcasts (relays per round, bit for bit)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "python-p2p-network_amd"))

import numpy as np  # noqa: E402

import bench  # noqa: E402
from p2pnetwork.gpu import GraphNetwork, PartitionedNetwork, make_sources  # noqa: E402
from p2pnetwork.gpu.network import PUSH_FORMS, STAT_FIELDS  # noqa: E402

XGMI_GBPS = 500.0  # per direction per GPU: 7 links x ~76 GB/s one way (MI355X_MICROARCH.md)


class NoTransport:
    """PartitionedNetwork's constructor wants a transport; the rounds here are driven by hand."""
    rows_total = rows_sent = 0

    def engine_stream(self):
        return None


def kernel_ms(net):
    return sum(v[0] for v in net.kernel_times().values())


def one_step(pns, W):
    import torch
    world = len(pns)
    R = 1 + W
    plane = pns[0]._plane
    rounds, per = [], []
    for pn in pns:
        pn.reset()
    while True:
        ks, stats = [], []
        for pn in pns:  # one rank at a time, each round finished before the next rank's starts
            k0 = kernel_ms(pn.net)
            st = pn.net.step()
            ks.append(kernel_ms(pn.net) - k0)
            stats.append(st)
        counts = [np.asarray(pn.net.exchange_pack_live(plane, pn._bufs[0]), dtype=np.int64) for pn in pns]
        sent = [int(c.sum()) * R * 8 for c in counts]
        recv = [int(sum(counts[p][q] for p in range(world) if p != q)) * R * 8 for q in range(world)]
        for q, pn in enumerate(pns):
            rbuf = pn._bufs[1]
            off = 0
            rc = np.zeros(world, dtype=np.int64)
            for p in range(world):
                if p == q:
                    continue
                n = int(counts[p][q])
                rc[p] = n
                if n:
                    so = int(np.concatenate([[0], np.cumsum(pns[p]._send_rows(plane))])[q])
                    rbuf[off * R:(off + n) * R].copy_(pns[p]._bufs[0][so * R:(so + n) * R])
                    off += n
            torch.cuda.synchronize()
            pn.net.exchange_unpack_live(plane, rbuf, rc)
        torch.cuda.synchronize()
        tot = {f: sum(int(getattr(s, f)) for s in stats) for f in STAT_FIELDS[2:]}
        rounds.append(tot)
        per.append({"kernel_ms": ks, "sent_B": sent, "recv_B": recv,
                    "forms": [PUSH_FORMS[s.push_form] if s.push_form < len(PUSH_FORMS) else s.push_form
                              for s in stats]})
        if tot["new_deliveries"] == 0 and stats[0].round > 0:
            break
    return rounds, per


def main():
    world = int(sys.argv[1])
    M = int(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    w = dict(bench.WORKLOADS["c4"])
    g = bench.build_graph(w)
    src = make_sources(g.V, w["M"], seed=1)[:M]
    W = (M + 63) // 64
    kw = dict(mode="gossip", fanout=3, gossip_seed=bench.GOSSIP_SEED, timing=True)
    with GraphNetwork(g, **kw) as one:
        one.broadcast(src)
        ref = [r.relays for r in one.run()]
    t0 = time.perf_counter()
    pns = [PartitionedNetwork(g, world, r, NoTransport(), overlap=False, **kw) for r in range(world)]
    for pn in pns:
        pn.broadcast(src)
    setup_s = time.perf_counter() - t0
    runs = []
    for s in range(steps):
        rounds, per = one_step(pns, W)
        relays = [r["relays"] for r in rounds]
        # round 0 of a partitioned rank counts only the origins it holds; the global round 0 is
        # the sum over ranks of their own origins' relays -- compare from round 1 on
        ok = relays[1:len(ref)] == ref[1:len(relays)] and sum(relays[1:]) == sum(ref[1:])
        kern = [max(p["kernel_ms"]) for p in per]
        xch = [max(max(p["sent_B"]), max(p["recv_B"])) / (XGMI_GBPS * 1e9) * 1e3 for p in per]
        runs.append({"relays_equal_one_engine": ok, "rounds": len(rounds),
                     "slowest_rank_kernel_ms": sum(kern), "exchange_ms_at_xgmi": sum(xch),
                     "projected_step_ms": sum(kern) + sum(xch),
                     "rank_kernel_ms_total": [sum(p["kernel_ms"][r] for p in per) for r in range(world)],
                     "exchange_GB_max_rank": sum(max(max(p["sent_B"]), max(p["recv_B"])) for p in per) / 1e9,
                     "per_round": per if s == steps - 1 else None})
    for pn in pns:
        pn.close()
    out = {"world": world, "broadcasts": M, "W": W, "setup_s": setup_s,
           "ghosts": [int(pn.part.V_local - 1 - (pn.part.hi - pn.part.lo)) for pn in pns],
           "fused_every_rank": all(any(f == "fused" for f in [x["forms"][r] for x in runs[-1]["per_round"]])
                                   for r in range(world)),
           "runs": runs}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
