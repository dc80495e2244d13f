"""bench.py's byte models (CPU): SURVEY.md 8(d)'s B_r, as the roofline's algorithmic bytes, and
the engine's per-kernel model beside it, on per-round counters from the numpy oracle."""
import types

import numpy as np
import pytest

import bench
from oracle import relay_oracle

FIELDS = ("new_deliveries", "relays", "active_vertices", "active_words", "wedges", "deg_active",
          "scatter_words", "touched_words", "push_form")


def rounds_of(ora_rounds, forms):
    out = []
    for r, f in zip(ora_rounds, forms):
        d = {k: int(r.get(k, 0)) for k in FIELDS if k != "push_form"}
        d["push_form"] = f
        out.append(types.SimpleNamespace(**d))
    return out


def gossip_rounds():
    rng = np.random.default_rng(3)
    V, d = 300, 6
    e = set()
    while len(e) < V * d // 2:
        a, b = (int(x) for x in rng.integers(0, V, 2))
        if a != b:
            e.add((min(a, b), max(a, b)))
    rows = [[] for _ in range(V)]
    for a, b in e:
        rows[a].append(b)
        rows[b].append(a)
    rowptr = np.zeros(V + 1, dtype=np.int64)
    rowptr[1:] = np.cumsum([len(r) for r in rows])
    colidx = np.concatenate([sorted(r) for r in rows]).astype(np.int32)
    src = rng.integers(0, V, 128).astype(np.int32)
    return relay_oracle.gossip(rowptr, colidx, src, 3, 0x5EED, 0, 0, 0).rounds


def test_survey_bytes_formula_per_round():
    ora = gossip_rounds()
    n = len(ora)
    rounds = rounds_of(ora, [bench.ATOMIC] * n)
    tot = bench.survey_bytes(rounds, "gossip")
    want = 0
    for i in range(1, n):
        p, r = ora[i - 1], ora[i]
        # B_r = 8 N_bitrelay(r-1) + 8 N_aw(r-1) + 4 sum deg(A_{r-1}) + 8 |A_{r-1}| + 24 N_nw(r)
        want += (8 * p["relays"] + 8 * p["active_words"] + 4 * p["deg_active"]
                 + 8 * p["active_vertices"] + 24 * r["active_words"])
    assert tot == want > 0


@pytest.mark.parametrize("pattern", ["all_atomic", "dense_middle", "update_edge_middle"])
def test_kernel_split_of_survey_bytes_is_a_partition(pattern):
    """Every round's B_r goes to exactly one kernel class (the one consuming its arrivals), so
    the per-kernel SURVEY bytes the roofline uses add up to the whole-step figure."""
    ora = gossip_rounds()
    n = len(ora)
    if pattern == "all_atomic":
        forms = [bench.ATOMIC] * n
    else:  # sparse, one edge-store round (or update + edge pushes in one pass), fused rounds,
        # back to sparse
        forms = [bench.ATOMIC] * n
        lo, hi = n // 3, 2 * n // 3
        forms[lo] = bench.EDGE if pattern == "dense_middle" else bench.UPDATE_EDGE
        for i in range(lo + 1, hi):
            forms[i] = bench.FUSED
    rounds = rounds_of(ora, forms)
    whole = bench.survey_bytes(rounds, "gossip")
    parts = {k: bench.survey_bytes_kernel(rounds, "gossip", k) for k in bench.KCLASS}
    assert sum(parts.values()) == whole
    if pattern == "dense_middle":
        assert parts["gossip_fused"] > 0 and parts["gossip_pull"] > 0 and parts["gossip_update"] > 0
    elif pattern == "update_edge_middle":
        # the update + push pass is timed as gossip_scatter_store: its round's B_r goes there
        p, r = ora[lo - 1], ora[lo]
        assert parts["gossip_scatter_store"] == (8 * p["relays"] + 8 * p["active_words"]
                                                 + 4 * p["deg_active"] + 8 * p["active_vertices"]
                                                 + 24 * r["active_words"]) > 0
        assert parts["gossip_fused"] > 0 and parts["gossip_pull"] > 0
    else:
        assert parts["gossip_update"] == whole


def test_flood_models_agree():
    """Flood: the engine's pull model is SURVEY's B_r term for term."""
    ora = gossip_rounds()
    rounds = rounds_of(ora, [0] * len(ora))
    for r in rounds:
        r.relays = r.wedges  # flood moves a frontier word per active word-edge
    mb = bench.model_bytes(rounds, "flood", 2)
    assert mb["flood_pull"] == bench.survey_bytes(rounds, "flood") == \
        bench.survey_bytes_kernel(rounds, "flood", "flood_pull")
