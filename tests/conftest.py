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
    """Golden fixture names; dynamic=True: only the ones with connection changes between
    rounds (dyn_*, which need updates_of), else only the static-topology ones."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f.startswith(prefix)
                  and f != "config1_tcp.npz" and f.startswith("dyn_") == dynamic)


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
