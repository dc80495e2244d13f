"""Per-round statistics and per-kernel device time of one workload (development aid).

    python tools/round_profile.py c4 [runs] [msgs] > gpurun_out/rounds_c4.json
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "python-p2p-network_amd"))

import bench  # noqa: E402
from p2pnetwork.gpu import GraphNetwork, make_sources  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c4"
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    w = dict(bench.WORKLOADS[wl])
    if len(sys.argv) > 3:
        w["M"] = int(sys.argv[3])
    g = bench.build_graph(w)
    src = make_sources(g.V, w["M"], seed=1)
    with GraphNetwork(g, mode=w["mode"], fanout=w["fanout"], gossip_seed=0x5EED, timing=True) as net:
        net.broadcast(src)
        net.run()
        out = []
        for i in range(runs):
            net.reset()
            t = time.perf_counter()
            rounds = []
            while True:
                k0 = net.kernel_times()
                st = net.step()
                k1 = net.kernel_times()
                d = st.as_dict()
                d["push_form"] = st.push_form
                d["kernel_ms"] = {k: k1[k][0] - k0[k][0] for k in k1}
                rounds.append(d)
                if not st.active:
                    break
            out.append({"wall_ms": (time.perf_counter() - t) * 1e3, "rounds": rounds})
    print(json.dumps({"workload": wl, "runs": out}))


if __name__ == "__main__":
    main()
