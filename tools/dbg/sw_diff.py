"""Debug: GPU gossip vs C oracle per round on a BA graph (first differing round / counter)."""
import sys, os
import numpy as np
sys.path[:0] = ["/root/repo", "/root/repo/python-p2p-network_amd"]
from oracle import coracle
from p2pnetwork.gpu import GraphNetwork, PeerGraph, make_sources
V, M = int(sys.argv[1]), int(sys.argv[2])
g = PeerGraph.barabasi_albert(V, 4, seed=5)
src = make_sources(g.V, M, seed=5)
with GraphNetwork(g, mode="gossip", fanout=3, gossip_seed=0x5EED) as net:
    net.broadcast(src)
    rounds = net.run()
    seen = net.seen_plane()
ora = coracle.run(g.rowptr, g.colidx, src, "gossip", 3, 0x5EED, record=False, want_seen=True)
keys = ("new_deliveries", "relays", "active_vertices", "active_words", "wedges", "deg_active", "scatter_words")
for i, (a, b) in enumerate(zip([r.as_dict() for r in rounds], ora.rounds)):
    bad = [k for k in keys if a[k] != b[k]]
    print(i, rounds[i].push_form, a["new_deliveries"], b["new_deliveries"], bad, flush=True)
    if bad:
        break
d = seen != ora.seen
print("mismatched words", int(d.sum()), "rows", int(d.any(1).sum()), "cols", np.nonzero(d.any(0))[0][:20])
