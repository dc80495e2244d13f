"""ctypes binding of libp2pgpu.so (the C-ABI in include/p2pgpu.h).

No PyTorch dependency.  The library is built in-tree (``make -C python-p2p-network_amd/csrc``
or ``__graft_entry__.build()``); if it is missing this module raises -- there is no CPU
fallback on the product path.
"""
import ctypes
import os

import numpy as np

LIB_NAME = "libp2pgpu.so"
# P2PG_LIB: load another build of the library (A/B comparisons of kernel variants)
LIB_PATH = os.environ.get("P2PG_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

MODE_FLOOD = 0
MODE_GOSSIP = 1
FLAG_RECORD = 1
FLAG_TIMING = 2
FLAG_NO_AUTOSTOP = 4
FLAG_LOCAL_GRAPH = 8
FLAG_RECEIVED = 16

# graph kinds of p2pg_graph_generate
GRAPH_RANDOM_REGULAR = 0
GRAPH_GNP = 1
GRAPH_BARABASI_ALBERT = 2
GRAPH_WATTS_STROGATZ = 3
GRAPH_RING_CHORDS = 4

ERRORS = {-1: "bad argument", -2: "bad state", -3: "HIP error", -4: "out of memory", -5: "bad graph"}


class P2PGError(RuntimeError):
    """Raised for any negative return code of the C-ABI (message from p2pg_last_error)."""


class Config(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32),
        ("fanout", ctypes.c_int32),
        ("gossip_seed", ctypes.c_uint64),
        ("churn_seed", ctypes.c_uint64),
        ("churn_threshold", ctypes.c_uint32),
        ("msg_id_base", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("device", ctypes.c_int32),
    ]


class RoundStatsC(ctypes.Structure):
    _fields_ = [
        ("round", ctypes.c_int32),
        ("active", ctypes.c_int32),
        ("new_deliveries", ctypes.c_uint64),
        ("relays", ctypes.c_uint64),
        ("active_vertices", ctypes.c_uint64),
        ("active_words", ctypes.c_uint64),
        ("wedges", ctypes.c_uint64),
        ("deg_active", ctypes.c_uint64),
        ("scatter_words", ctypes.c_uint64),
        ("touched_words", ctypes.c_uint64),
        ("push_form", ctypes.c_int32),
        ("received_exact", ctypes.c_int32),
        ("received", ctypes.c_uint64),
    ]


# every symbol declared in include/p2pgpu.h, with (restype, argtypes)
_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_PP = ctypes.POINTER(ctypes.c_void_p)
SIGNATURES = {
    "p2pg_graph_generate": (ctypes.c_int, [_I32, _I64, ctypes.c_double, ctypes.c_double, _U64, _PP]),
    "p2pg_graph_from_edges": (ctypes.c_int, [_I64, _I64, _P, _P, _PP]),
    "p2pg_graph_info": (ctypes.c_int, [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "p2pg_graph_arrays": (ctypes.c_int, [_P, _PP, _PP]),
    "p2pg_graph_free": (None, [_P]),
    "p2pg_make_sources": (ctypes.c_int, [_I64, _I32, _U64, _U32, _P]),
    "p2pg_philox4x32_10": (None, [_P, _P, _P]),
    "p2pg_gossip_targets": (ctypes.c_int, [_U32, _U32, _U32, _U32, _I32, _U64, _P]),
    "p2pg_churn_lost": (ctypes.c_int, [_U32, _U32, _U32, _U32, _U64]),
    "p2pg_create": (ctypes.c_int, [ctypes.POINTER(Config), _PP]),
    "p2pg_load_csr": (ctypes.c_int, [_P, _I64, _P, _P]),
    "p2pg_set_sources": (ctypes.c_int, [_P, _I32, _P]),
    "p2pg_reset": (ctypes.c_int, [_P]),
    "p2pg_step": (ctypes.c_int, [_P, ctypes.POINTER(RoundStatsC)]),
    "p2pg_run": (ctypes.c_int, [_P, _I32, _P, ctypes.POINTER(_I32)]),
    "p2pg_get_new_deliveries": (ctypes.c_int, [_P, _I64, _P, _P, _P, _P, ctypes.POINTER(_I64)]),
    "p2pg_get_sends": (ctypes.c_int, [_P, _I64, _P, _P, _P, _P, ctypes.POINTER(_I64)]),
    "p2pg_drop_relays": (ctypes.c_int, [_P, _I64, _P, _P]),
    "p2pg_read_planes": (ctypes.c_int, [_P, _P, _P, _P]),
    "p2pg_read_seen_word": (ctypes.c_int, [_P, _I32, _P]),
    "p2pg_kernel_times": (ctypes.c_int, [_P, _P, _P]),
    "p2pg_set_timed_classes": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "p2pg_set_global_ids": (ctypes.c_int, [_P, _P]),
    "p2pg_set_exchange": (ctypes.c_int, [_P, _I64, _P, _I64, _P]),
    "p2pg_set_ghost_senders": (ctypes.c_int, [_P, _P, _P]),
    "p2pg_exchange_pack": (ctypes.c_int, [_P, _I32, _P]),
    "p2pg_exchange_unpack": (ctypes.c_int, [_P, _I32, _P]),
    "p2pg_set_exchange_segments": (ctypes.c_int, [_P, _I32, _P, _P]),
    "p2pg_exchange_pack_live": (ctypes.c_int, [_P, _I32, _P, _P]),
    "p2pg_exchange_unpack_live": (ctypes.c_int, [_P, _I32, _P, _P]),
    "p2pg_set_exchange_buffer": (ctypes.c_int, [_P, _I32, _P]),
    "p2pg_step_begin": (ctypes.c_int, [_P]),
    "p2pg_step_end": (ctypes.c_int, [_P, ctypes.POINTER(RoundStatsC)]),
    "p2pg_set_stream": (ctypes.c_int, [_P, _P]),
    "p2pg_device_philox": (ctypes.c_int, [_P, _I32, _P, _P, _P]),
    "p2pg_update_edges": (ctypes.c_int, [_P, _I64, _P, _I64, _P]),
    "p2pg_snapshot_size": (ctypes.c_int, [_P, ctypes.POINTER(_I64)]),
    "p2pg_snapshot": (ctypes.c_int, [_P, _P, _I64]),
    "p2pg_restore": (ctypes.c_int, [_P, _P, _I64]),
    "p2pg_last_error": (ctypes.c_char_p, [_P]),
    "p2pg_global_error": (ctypes.c_char_p, []),
    "p2pg_destroy": (None, [_P]),
}

_lib = None


def _share_hip_runtime():
    """Use PyTorch's HIP runtime when PyTorch is installed.

    libp2pgpu.so links libamdhip64.so.7 from /opt/rocm; PyTorch ships its own build with the
    same soname, and the first one loaded serves the whole process.  If ours came first,
    PyTorch's later HIP initialisation fails ("No HIP GPUs are available"), so before loading
    the engine the torch copy is preloaded (without importing torch).  Both the partitioned
    path (RCCL via torch.distributed) and callers mixing torch tensors then share one runtime.
    P2PG_HIP_RUNTIME=system keeps /opt/rocm's runtime (processes that never use torch)."""
    if os.environ.get("P2PG_HIP_RUNTIME", "") == "system":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(p):
            ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
            return


def lib():
    """Load (once) and return the bound library; raises P2PGError if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise P2PGError(
                f"{LIB_PATH} is not built: run `make -C python-p2p-network_amd/csrc` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        _share_hip_runtime()
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc, engine=None):
    if rc is not None and rc < 0:
        L = lib()
        msg = L.p2pg_last_error(engine) if engine else L.p2pg_global_error()
        raise P2PGError(f"{ERRORS.get(rc, rc)}: {msg.decode(errors='replace') if msg else ''}")
    return rc


def ptr(a):
    """data pointer of a C-contiguous numpy array (None for None)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def philox_host(ctr, key):
    """Host Philox4x32-10 of the library (one counter)."""
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().p2pg_philox4x32_10(ptr(c), ptr(k), ptr(out))
    return out
