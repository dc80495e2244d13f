"""Oracle digests of the full-size config-4 and config-5 seen planes (test infrastructure).

Runs the C oracle (oracle/relay_oracle.c, itself pinned to the reference-harness fixtures by
tests/test_oracle_golden.py) once per 64-message word on the deterministic BASELINE graphs, IN
THIS CONTAINER, and writes a small fixture per config:

* ``csr``       -- xxh3-128 of the generated rowptr and colidx (the GPU box regenerates the
                   graph with the same generator and seed; the digest proves it is this graph);
* ``word_dig``  -- [64, 16] uint8: xxh3-128 of word w's seen column (uint64 [V], messages
                   64w .. 64w+63) of the oracle's 64-message run of those messages;
* ``rounds``    -- [64, R, 7] uint64: the oracle's per-round counters of each word's run
                   (coracle.KEYS order), zero-padded.

The GPU tests then hold the 4096-message run's 64 seen columns (p2pg_read_seen_word) to these
digests and its additive per-round counters to the sums -- the whole plane pinned to the oracle
at no oracle cost on the GPU box.  Config 4: 10M-peer BA m=4, gossip k=3, seed 0x5EED.
Config 5: 100M-peer WS k=8 beta=0.1, churn 0.05 (seed 0xC0FFEE), flood.  (bench.py's seeds.)

Usage:  python tests/golden/make_plane_digests.py [c4|c5]     (~10 min / ~40 min on 8 cores)
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "python-p2p-network_amd"))

from oracle import coracle  # noqa: E402
from p2pnetwork.gpu import PeerGraph, make_sources  # noqa: E402
from p2pnetwork.gpu.network import churn_threshold  # noqa: E402

MAX_ROUNDS = 128


def digest(a):
    import xxhash
    return np.frombuffer(xxhash.xxh3_128_digest(np.ascontiguousarray(a)), dtype=np.uint8)


def csr_digest(g):
    import xxhash
    h = xxhash.xxh3_128()
    h.update(np.ascontiguousarray(g.rowptr, dtype=np.int64))
    h.update(np.ascontiguousarray(g.colidx, dtype=np.int32))
    return np.frombuffer(h.digest(), dtype=np.uint8)


def make(name, g, src, **kw):
    W = len(src) // 64
    dig = np.zeros((W, 16), dtype=np.uint8)
    rounds = np.zeros((W, MAX_ROUNDS, len(coracle.KEYS)), dtype=np.uint64)
    for w in range(W):
        t = time.time()
        ora = coracle.run(g.rowptr, g.colidx, src[64 * w:64 * (w + 1)], record=False, want_seen=True,
                          msg_id_base=64 * w, **kw)
        dig[w] = digest(ora.seen[:, 0])
        for i, r in enumerate(ora.rounds):
            rounds[w, i] = [r[k] for k in coracle.KEYS]
        print(f"{name} word {w}: {len(ora.rounds)} rounds, {time.time() - t:.1f} s", flush=True)
        del ora
    out = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(out, csr=csr_digest(g), word_dig=dig, rounds=rounds, V=np.int64(g.V),
                        M=np.int64(len(src)))
    print(f"{name}: -> {out} ({os.path.getsize(out)} B)")


def main():
    which = sys.argv[1:] or ["c4", "c5"]
    if "c4" in which:
        g = PeerGraph.barabasi_albert(10_000_000, 4, seed=1)
        make("plane_c4_ba10m_gossip", g, make_sources(g.V, 4096, seed=1), mode="gossip", fanout=3,
             gossip_seed=0x5EED)
        del g
    if "c5" in which:
        g = PeerGraph.watts_strogatz(100_000_000, 8, 0.1, seed=1)
        make("plane_c5_ws100m_churn", g, make_sources(g.V, 4096, seed=1), mode="flood",
             churn_threshold=churn_threshold(0.05), churn_seed=0xC0FFEE)


if __name__ == "__main__":
    main()
