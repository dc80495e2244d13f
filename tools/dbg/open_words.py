"""Open words per unsaturated peer at the start of each round of config 4 (the sizing question
of a compacted several-peers-per-wave form of the light dense rounds), and the
arrival union: the words of the OR of the active neighbours' active-word masks (the words a
peer's gathers can bring), per visited non-hub peer.

A word of a peer's seen row is open while any of its 64 messages is still unseen; the fused
kernel visits every unsaturated non-hub peer with a whole 64-lane wave, whatever the number
of open words.  Steps the bench workload round by round, reads the seen plane after each
round and prints, per round, the visited peers and the share whose open words (and whose
arrival union) fit 8 / 16 / 32 lanes.

    python tools/dbg/open_words.py [first_round] [last_round]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "python-p2p-network_amd"))


def main():
    import bench
    from p2pnetwork.gpu import GraphNetwork, make_sources
    lo = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    hi = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    w = bench.WORKLOADS["c4"]
    g = bench.build_graph(w)
    deg = np.diff(g.rowptr)
    hub = deg > 512
    src = make_sources(g.V, w["M"], seed=1)
    net = GraphNetwork(g, mode="gossip", fanout=w["fanout"], gossip_seed=bench.GOSSIP_SEED)
    net.broadcast(src)
    print(f"V {g.V} hubs {int(hub.sum())} deg<=64 {float((deg <= 64).mean()):.4f}", flush=True)
    prev = None
    for r in range(hi + 1):
        st = net.step()
        if r + 2 < lo:
            continue
        t0 = time.perf_counter()
        s = net.seen_plane()
        if r + 1 < lo:
            prev = s
            continue
        openw = (s != np.uint64(0xFFFFFFFFFFFFFFFF)).sum(axis=1)
        # active-word masks of round r (the words whose seen bits changed), OR over neighbours
        aw = np.packbits(s != prev, axis=1, bitorder="little").view(np.uint64)[:, 0]
        prev = s
        un = np.bitwise_count(np.bitwise_or.reduceat(aw[g.colidx], g.rowptr[:-1]))
        vis = (openw > 0) & ~hub
        ov = openw[vis]
        n = int(vis.sum())
        fr = [float((ov <= k).mean()) if n else 0.0 for k in (8, 16, 32)]
        small = vis & (deg <= 64)
        uv = un[vis]
        fu = [float((uv <= k).mean()) if n else 0.0 for k in (8, 16, 32)]
        print(f"round {r + 1:3d} (after {r}: new {st.new_deliveries:>11d})  visited {n:>9d}  "
              f"open mean {float(ov.mean()) if n else 0:5.1f}  p50 {int(np.median(ov)) if n else 0:2d}  "
              f"<=8 {fr[0]:.3f} <=16 {fr[1]:.3f} <=32 {fr[2]:.3f}  "
              f"(deg<=64 & <=16: {float(((openw <= 16) & small).sum() / max(n, 1)):.3f})  "
              f"union mean {float(uv.mean()) if n else 0:5.1f} <=8 {fu[0]:.3f} <=16 {fu[1]:.3f} "
              f"<=32 {fu[2]:.3f} empty {float((uv == 0).mean()) if n else 0:.3f}  "
              f"{time.perf_counter() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
