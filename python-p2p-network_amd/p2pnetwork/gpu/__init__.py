"""p2pnetwork.gpu -- MI355X broadcast/relay engine for p2pnetwork's flood-relay hot path.

    from p2pnetwork.gpu import PeerGraph, GraphNetwork, make_sources
    g = PeerGraph.gnp(1_000_000, 16, seed=1)
    with GraphNetwork(g, mode="flood") as net:
        net.broadcast(make_sources(g.V, 4096, seed=1))
        rounds = net.run()

The HIP engine is reached through ctypes (``_lib``); there is no CPU fallback.
"""
from ._lib import P2PGError, LIB_PATH
from .graph import PeerGraph, make_sources
from .network import GraphNetwork, RoundStats, Deliveries, churn_threshold
from .partition import VertexPartition, PartitionedNetwork, TorchTransport
from .compat import SimNode, SimConnection, CompatNetwork
from . import wire

__all__ = ["P2PGError", "LIB_PATH", "PeerGraph", "make_sources", "GraphNetwork", "RoundStats",
           "Deliveries", "churn_threshold", "VertexPartition", "PartitionedNetwork", "TorchTransport",
           "SimNode", "SimConnection", "CompatNetwork", "wire"]
