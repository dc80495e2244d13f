import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "python-p2p-network_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def golden_cases(prefix="", dynamic=False):
    """Golden relay fixtures (hop / parent / per-round relays from the reference harness);
    dynamic=True: only the ones with connection changes between rounds (dyn_*, which need
    updates_of), else only the static-topology ones.  The real-TCP fixtures (config1_tcp,
    tcp*) hold reachability only: tcp_cases()."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f.startswith(prefix)
                  and not f.startswith(("config1_tcp", "tcp", "app_", "plane_"))
                  and f.startswith("dyn_") == dynamic)


def app_cases():
    """Hook-semantics fixtures (app_*): Node apps of tests/compat_apps.py run on the reference's
    own Node objects -- every node_message call in order, every node's counters."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f.startswith("app_"))


def tcp_cases():
    """Real localhost-TCP runs of reference Nodes: reachability per (peer, msg) + relays."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz")
                  and f.startswith(("config1_tcp", "tcp")))


def wire_cases():
    """Harness runs with the bytes every connection carried per round (wire_*)."""
    return golden_cases("wire_")


def fixture_streams(z):
    """{round: {(sender, receiver): bytes}} of a wire_* fixture."""
    out = {}
    blob = z["s_blob"].tobytes()
    off = z["s_off"]
    for i, (r, a, b) in enumerate(zip(z["s_round"], z["s_sender"], z["s_receiver"])):
        out.setdefault(int(r), {})[(int(a), int(b))] = blob[off[i]:off[i + 1]]
    return out


def deliveries_from_planes(hop, parent, r):
    """Round r's first receipts (Deliveries, sorted by (peer, msg)) from hop/parent planes."""
    import numpy as np
    from p2pnetwork.gpu.network import Deliveries
    vs, ms = np.nonzero(hop == r)
    return Deliveries(vs.astype(np.int32), ms.astype(np.int32), np.full(len(vs), r, np.int32),
                      parent[vs, ms].astype(np.int32))


def updates_of(z):
    """{round r: (add_pairs, remove_pairs)} of a dyn_* fixture (changes after round r)."""
    out = {}
    for i, r in enumerate(z["upd_rounds"]):
        a = z["upd_add"][z["upd_add_off"][i]:z["upd_add_off"][i + 1]]
        d = z["upd_remove"][z["upd_remove_off"][i]:z["upd_remove_off"][i + 1]]
        out[int(r)] = (a, d)
    return out


def load_golden(name):
    import numpy as np
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def trim_zeros(a):
    import numpy as np
    a = np.asarray(a, dtype=np.int64)
    nz = np.nonzero(a)[0]
    return a[: nz[-1] + 1] if len(nz) else a[:0]
