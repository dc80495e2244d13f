"""ctypes wrapper of oracle/_build/liboracle.so (ORACLE -- test infrastructure only; see
oracle/__init__.py).  Same results as oracle.relay_oracle, in C with OpenMP, so it can also
serve as bench.py's timed CPU baseline ("kind": "port")."""
import ctypes
import os

import numpy as np

from .relay_oracle import RelayResult

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
KEYS = ("new_deliveries", "relays", "active_vertices", "active_words", "wedges", "deg_active",
        "scatter_words")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} not built: run `make -C oracle`")
        L = ctypes.CDLL(LIB)
        P, I32, I64, U32, U64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64
        L.oracle_flood.argtypes = [I64, P, P, I32, P, U32, U64, I32, P, P, P, P, P]
        L.oracle_gossip.argtypes = [I64, P, P, I32, P, I32, U64, U32, U32, U64, I32, P, P, P, P, P]
        L.oracle_flood.restype = L.oracle_gossip.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def run(rowptr, colidx, src, mode="flood", fanout=3, gossip_seed=0, msg_id_base=0,
        churn_threshold=0, churn_seed=0, record=True, max_rounds=100000, want_seen=False):
    """Oracle run; the result carries .seen ([V][W] uint64 seen sets) when want_seen."""
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    colidx = np.ascontiguousarray(colidx, dtype=np.int32)
    src = np.ascontiguousarray(src, dtype=np.int32)
    V, M = len(rowptr) - 1, len(src)
    stats = np.zeros((max_rounds, 8), dtype=np.uint64)
    n = ctypes.c_int32()
    hop = np.zeros((V, M), dtype=np.int32) if record else None
    par = np.zeros((V, M), dtype=np.int32) if record else None
    seen = np.zeros((V, (M + 63) // 64), dtype=np.uint64) if want_seen else None
    if mode == "flood":
        rc = lib().oracle_flood(V, _p(rowptr), _p(colidx), M, _p(src), churn_threshold, churn_seed,
                                max_rounds, _p(stats), ctypes.byref(n), _p(hop), _p(par), _p(seen))
    else:
        rc = lib().oracle_gossip(V, _p(rowptr), _p(colidx), M, _p(src), fanout, gossip_seed, msg_id_base,
                                 churn_threshold, churn_seed, max_rounds, _p(stats), ctypes.byref(n),
                                 _p(hop), _p(par), _p(seen))
    if rc:
        raise RuntimeError(f"oracle returned {rc}")
    rounds = [dict(round=i, **{k: int(stats[i, j]) for j, k in enumerate(KEYS)}) for i in range(n.value)]
    res = RelayResult(hop, par, rounds)
    res.seen = seen
    return res
