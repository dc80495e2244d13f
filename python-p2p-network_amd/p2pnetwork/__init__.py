"""p2pnetwork (MI355X build): the flood/gossip relay hot path of pj8912/python-p2p-network,
re-implemented as a whole-graph HIP engine.  Only the ``gpu`` subpackage lives here; the
reference's TCP Node/NodeConnection layer is out of scope.
"""
__all__ = ["gpu"]
