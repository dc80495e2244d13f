"""Probe: does torch's HIP init survive libp2pgpu.so (linked to /opt/rocm's libamdhip64) being
loaded first?  Both runtimes share the soname libamdhip64.so.7, so the first one loaded wins."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "python-p2p-network_amd"))
order = sys.argv[1]
if order == "torch-first":
    import torch
from p2pnetwork.gpu import GraphNetwork, PeerGraph
net = GraphNetwork(PeerGraph.ring_chords(10, 3))
net.broadcast([0])
print("rounds", len(net.run()))
import torch
torch.cuda.init()
x = torch.ones(4, device="cuda:0")
print(order, "torch ok", float(x.sum()))
with open("/proc/self/maps") as f:
    print(sorted({l.split()[-1] for l in f if "libamdhip64" in l}))
