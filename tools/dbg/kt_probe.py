import sys, os, time
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/python-p2p-network_amd')
import bench
from p2pnetwork.gpu import GraphNetwork, make_sources
w = bench.WORKLOADS['c3']
g = bench.build_graph(w)
src = make_sources(g.V, w['M'], seed=1)
net = GraphNetwork(g, mode='flood', timing=True)
net.broadcast(src)
for i in range(3):
    net.reset(); r = net.run()
    kt = net.kernel_times()
    print(i, len(r), {k: (round(v[0], 3), v[1]) for k, v in kt.items() if v[1]}, flush=True)
