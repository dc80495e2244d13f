"""Philox4x32-10 restatement in numpy (ORACLE -- test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker.  The product path (python-p2p-network_amd/) never imports oracle/.

Algorithm: Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3" (SC'11),
Random123 philox4x32 with R = 10; constants as in /opt/rocm/include/rocrand/
rocrand_philox4x32_10.h:62-65.  Pinned by the Random123 known-answer vectors in
tests/test_philox.py.  The gossip pick rule (Floyd + Lemire) and the
churn rule restate SURVEY.md A.3 / A.4; the reference library has no randomised relay, so
these are the build's own definitions, pinned by the golden fixtures generated through the
reference Node objects (tests/golden/make_golden.py).
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint64(0x9E3779B9)
W1 = np.uint64(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)
S32 = np.uint64(32)

TAG_SRC = 0x00535243
TAG_GSP = 0x00475350
TAG_CHN = 0x0043484E


def _u(x):
    return np.asarray(x, dtype=np.uint64) & MASK


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10. Inputs broadcast; returns four uint64 arrays of 32-bit values."""
    c0, c1, c2, c3 = _u(c0), _u(c1), _u(c2), _u(c3)
    k0, k1 = _u(k0), _u(k1)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> S32) ^ c1 ^ k0) & MASK, p1 & MASK, ((p0 >> S32) ^ c3 ^ k1) & MASK, p0 & MASK
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return c0, c1, c2, c3


def lemire32(x, n):
    return (_u(x) * np.asarray(n, dtype=np.uint64)) >> S32


def make_sources(V, M, seed, msg_id_base=0):
    """src[m] = lemire32(philox(key=(seed_lo, seed_hi ^ 'SRC'), ctr=(base+m,0,0,0)).x, V)."""
    m = np.arange(M, dtype=np.uint64) + np.uint64(msg_id_base)
    k0 = np.uint64(seed & 0xFFFFFFFF)
    k1 = np.uint64(((seed >> 32) & 0xFFFFFFFF) ^ TAG_SRC)
    x, _, _, _ = philox4x32_10(m, 0, 0, 0, k0, k1)
    return lemire32(x, V).astype(np.int32)


def gossip_picks(rnd, peer, msg, n, k, seed):
    """k distinct indices in [0, n) per (round, peer, msg) row, Floyd's algorithm with Lemire
    reduction; draw i uses word i%4 of Philox block i//4 with ctr=(round, peer, msg,
    'GSP' | blk << 24).  Rows need n > k.  Returns int64 [N, k] in draw order."""
    rnd, peer, msg, n = np.broadcast_arrays(np.asarray(rnd), np.asarray(peer), np.asarray(msg), np.asarray(n))
    N = rnd.size
    out = np.zeros((N, k), dtype=np.int64)
    k0 = np.uint64(seed & 0xFFFFFFFF)
    k1 = np.uint64((seed >> 32) & 0xFFFFFFFF)
    words = None
    for i in range(k):
        if i % 4 == 0:
            words = philox4x32_10(rnd.ravel(), peer.ravel(), msg.ravel(),
                                  np.uint64(TAG_GSP | ((i // 4) << 24)), k0, k1)
        jmax = n.ravel().astype(np.int64) - k + i
        t = lemire32(words[i % 4], jmax + 1).astype(np.int64)
        dup = np.zeros(N, dtype=bool)
        for q in range(i):
            dup |= out[:, q] == t
        out[:, i] = np.where(dup, jmax, t)
    return out


def churn_dropped(rnd, a, b, threshold, seed):
    """Send over undirected edge {a,b} in round rnd is lost iff philox(...).x < threshold."""
    a = np.asarray(a, dtype=np.int64)
    b = np.asarray(b, dtype=np.int64)
    if threshold == 0:
        return np.zeros(np.broadcast(a, b).shape, dtype=bool)
    lo = np.minimum(a, b)
    hi = np.maximum(a, b)
    k0 = np.uint64(seed & 0xFFFFFFFF)
    k1 = np.uint64((seed >> 32) & 0xFFFFFFFF)
    x, _, _, _ = philox4x32_10(rnd, lo, hi, TAG_CHN, k0, k1)
    return x < np.uint64(threshold)
