"""Philox4x32-10 known-answer tests (Random123 kat_vectors) for the
numpy oracle restatement and the library's host implementation; the GPU twin is in
test_gpu_parity.py."""
import numpy as np
import pytest

from oracle import philox

KATS = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", KATS)
def test_oracle_philox_kat(ctr, key, want):
    got = philox.philox4x32_10(*ctr, *key)
    assert tuple(int(x) for x in got) == want


@pytest.mark.parametrize("ctr,key,want", KATS)
def test_library_host_philox_kat(ctr, key, want):
    from p2pnetwork.gpu import _lib
    assert tuple(int(x) for x in _lib.philox_host(ctr, key)) == want


def test_vectorised_matches_scalar():
    rng = np.random.default_rng(0)
    c = rng.integers(0, 2**32, size=(4, 50), dtype=np.uint64)
    k = rng.integers(0, 2**32, size=2, dtype=np.uint64)
    vec = philox.philox4x32_10(*c, *k)
    from p2pnetwork.gpu import _lib
    for i in range(50):
        host = _lib.philox_host(c[:, i], k)
        assert tuple(int(v[i]) for v in vec) == tuple(int(x) for x in host)


def test_gossip_picks_distinct_and_in_range():
    n = np.array([4, 5, 8, 100, 13000] * 40)
    pk = philox.gossip_picks(3, np.arange(200), np.arange(200) * 7, n, 3, 0xABCDEF)
    assert pk.shape == (200, 3)
    assert (pk >= 0).all() and (pk < n[:, None]).all()
    for row in pk:
        assert len(set(row.tolist())) == 3
    # k > 4 uses a second Philox block
    pk6 = philox.gossip_picks(0, np.arange(50), 0, 10, 6, 1)
    for row in pk6:
        assert len(set(row.tolist())) == 6


def test_sources_library_matches_oracle():
    from p2pnetwork.gpu import make_sources
    for V, M, seed, base in [(1000, 64, 1, 0), (10_000_000, 4096, 7, 4096), (3, 10, 2**40 + 5, 9)]:
        assert np.array_equal(make_sources(V, M, seed, base), philox.make_sources(V, M, seed, base))


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 7])
def test_library_gossip_targets_match_oracle(k):
    """p2pg_gossip_targets (the host twin of the device pushes; k <= 4 through the folded-round
    Philox of philox_pick / gossip_picks_k, which the dense pushes use) == the oracle's picks."""
    import ctypes
    from p2pnetwork.gpu import _lib
    rng = np.random.default_rng(k)
    n = 300
    rnd = rng.integers(0, 60, n)
    peer = rng.integers(0, 2**32, n, dtype=np.uint64)
    msg = rng.integers(0, 2**32, n, dtype=np.uint64)
    deg = rng.integers(k + 1, 20000, n)
    seed = int(rng.integers(0, 2**63))
    want = philox.gossip_picks(rnd, peer, msg, deg, k, seed)
    out = np.zeros(16, dtype=np.uint32)
    for i in range(n):
        got = _lib.lib().p2pg_gossip_targets(int(rnd[i]), int(peer[i]), int(msg[i]), int(deg[i]), k,
                                             seed, out.ctypes.data_as(ctypes.c_void_p))
        assert got == k
        assert out[:k].tolist() == [int(x) for x in want[i]], i
