"""CPU-side checks of the C-ABI boundary: libp2pgpu.so loads, exports every symbol that
include/p2pgpu.h declares, host-side entry points work without a GPU, and the engine fails
loudly (no silent CPU fallback) when no HIP device is visible."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO


def header_symbols():
    text = open(os.path.join(REPO, "include", "p2pgpu.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(p2pg_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from p2pnetwork.gpu import _lib
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    # and the ctypes signature table covers exactly the header
    assert sorted(_lib.SIGNATURES) == syms


def test_struct_layouts():
    from p2pnetwork.gpu import _lib
    assert ctypes.sizeof(_lib.Config) == 40
    assert ctypes.sizeof(_lib.RoundStatsC) == 88


def test_graph_generators_are_simple_undirected_and_deterministic():
    from p2pnetwork.gpu import PeerGraph
    for g in (PeerGraph.random_regular(500, 6, seed=3), PeerGraph.gnp(2000, 10, seed=4),
              PeerGraph.barabasi_albert(3000, 4, seed=5), PeerGraph.watts_strogatz(2000, 8, 0.1, seed=6),
              PeerGraph.ring_chords(10, 3)):
        g.validate()
    a = PeerGraph.barabasi_albert(3000, 4, seed=5)
    b = PeerGraph.barabasi_albert(3000, 4, seed=5)
    assert np.array_equal(a.rowptr, b.rowptr) and np.array_equal(a.colidx, b.colidx)
    assert set(PeerGraph.random_regular(500, 6, seed=3).degree()) == {6}
    ba = PeerGraph.barabasi_albert(3000, 4, seed=5)
    assert ba.degree().min() >= 4 and ba.n_edges == 10 + 4 * (3000 - 5)


def test_from_edges_drops_self_loops_and_duplicates():
    from p2pnetwork.gpu import PeerGraph
    g = PeerGraph.from_edges(5, [(0, 1), (1, 0), (2, 2), (3, 4), (4, 3), (0, 1)])
    assert g.n_edges == 2
    assert list(g.neighbours(0)) == [1] and list(g.neighbours(2)) == []


def test_invalid_graph_rejected():
    from p2pnetwork.gpu import PeerGraph
    with pytest.raises(ValueError):
        PeerGraph(np.array([0, 1, 1]), np.array([1]))  # not symmetric
    with pytest.raises(ValueError):
        PeerGraph(np.array([0, 1, 2]), np.array([0, 0]))  # self loop


def test_engine_create_without_gpu_fails_loudly():
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    from p2pnetwork.gpu import GraphNetwork, P2PGError, PeerGraph
    with pytest.raises(P2PGError, match="no HIP device"):
        GraphNetwork(PeerGraph.ring_chords(10, 3))
