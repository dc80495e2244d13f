"""ORACLE -- test infrastructure only.

CPU restatements of the reference relay semantics (pj8912/python-p2p-network).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import, call, link or execute
anything under oracle/, and only as the checker (or the timed CPU baseline), never as the
thing measured or shipped.  The product package python-p2p-network_amd/p2pnetwork/gpu never
imports it and fails loudly when its HIP library is missing.
"""
