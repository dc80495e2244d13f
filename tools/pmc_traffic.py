"""HBM traffic per launch of each relay kernel class from rocprofv3 PMC passes, calibrated.

    python tools/pmc_traffic.py CAL_DIR RUN_DIR WORKLOAD OUT_JSON [BUILD_SHA]

CAL_DIR: FETCH_SIZE / WRITE_SIZE passes over tools/microbench/atomics (known payloads:
seq_read, row_read, row_store of 5.12 GB each) -> bytes-per-counter-unit for 16 B/lane streams,
8 B/lane random 512 B row reads and row stores (MI355X_MICROARCH.md: FETCH_SIZE under-counts
wide streaming reads by 2x on gfx950; other widths must be calibrated).  RUN_DIR: the same two
passes over `bench.py --steps 1 --warmup 0 --no-cpu-baseline`.  The kernel rows of RUN_DIR are
converted with the row-read / row-store factors (the relay kernels move 512 B rows)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KNOWN = 10_000_000 * 512  # bytes per launch of the calibration kernels


def passes(d):
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "pass*", "*counter_collection.csv"))):
        rows += list(csv.DictReader(open(f)))
    return rows


def per_dispatch(rows):
    out = defaultdict(dict)
    for r in rows:
        k = (r["Kernel_Name"], int(r["Dispatch_Id"]))
        out[k][r["Counter_Name"]] = out[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        out[k]["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return out


def calib(d):
    f = defaultdict(list)
    for (name, _), c in per_dispatch(passes(d)).items():
        for key in ("seq_read", "row_read", "row_store"):
            if name.startswith(key) or f"{key}(" in name:
                if "FETCH_SIZE" in c:
                    f[key + ":fetch"].append(KNOWN / (c["FETCH_SIZE"] * 1024))
                if "WRITE_SIZE" in c:
                    f[key + ":write"].append(KNOWN / max(c["WRITE_SIZE"] * 1024, 1))
    return {k: sorted(v)[len(v) // 2] for k, v in f.items()}


def cls(name):
    """rocprof kernel name -> bench.py timer class (include/p2pgpu.h P2PG_KCLASS_N)."""
    tmpl = name.split("<", 1)[1].split(">(")[0] if "<" in name else ""
    targs = [t.strip() for t in tmpl.split(",")] if tmpl else []
    if "k_gossip_fused_grouped" in name:
        # <CHURN, K, LW, PO, PL>: push-only = the store pushes, pull-only = the last dense pull
        po = len(targs) > 3 and targs[3] == "true"
        pl = len(targs) > 4 and targs[4] == "true"
        return "gossip_scatter_store" if po else "gossip_pull" if pl else "gossip_fused"
    if "k_gossip_fused" in name:
        # <CHURN, K, MODE, HALF>: MODE 1 push-only / 2 update+push (timed with the store pushes),
        # 3 pull-only (timed as the last dense round's pull), 0 the fused round
        mode = targs[2] if len(targs) > 2 else "0"
        return {"1": "gossip_scatter_store", "2": "gossip_scatter_store",
                "3": "gossip_pull"}.get(mode, "gossip_fused")
    if "k_wide_zero" in name or "k_wide_push" in name:
        return "gossip_fused"  # (the hub pushes ride in the fused rounds' timed launch group)
    if any(x in name for x in ("k_sparse_words", "k_chunk_scan", "k_sparse_push", "k_touched_bits")):
        return "gossip_scatter_atomic"
    if "k_gossip_scatter" in name:
        return "gossip_scatter_store" if tmpl.rstrip().endswith("true") else "gossip_scatter_atomic"
    if "k_pull" in name:
        return "gossip_pull" if tmpl.rstrip().endswith("true") else "flood_pull"
    if "k_gossip_update" in name:
        return "gossip_update"
    if "k_seed" in name or "k_zero_rows" in name:
        return "seed"
    if "k_record" in name:
        return "record"
    return None


def main():
    cal_dir, run_dir, wl, out = sys.argv[1:5]
    cal = calib(cal_dir)
    rf = cal.get("row_read:fetch", 2.0)
    wf = cal.get("row_store:write", 1.0)
    agg = defaultdict(lambda: {"fetch": 0.0, "write": 0.0, "n": 0, "ns": 0})
    for (name, _), c in per_dispatch(passes(run_dir)).items():
        k = cls(name)
        if not k:
            continue
        a = agg[k]
        a["fetch"] += c.get("FETCH_SIZE", 0.0) * 1024 * rf
        a["write"] += c.get("WRITE_SIZE", 0.0) * 1024 * wf
        # helper kernels (hub pull partial/finalize, hub pushes, sparse-push list builders) ride
        # in the same timed launch group as their main kernel: count launches of the main one
        helper = any(x in name for x in ("k_pull_hub", "k_wide_", "k_sparse_words", "k_chunk_scan",
                                         "k_touched_bits"))
        a["n"] += 1 if ("FETCH_SIZE" in c and not helper) else 0
        a["ns"] += c["ns"] if "FETCH_SIZE" in c else 0
    res = {"workload": wl, "build_sha": sys.argv[5] if len(sys.argv) > 5 else None,
           "calibration": cal, "source": run_dir, "kernels": {}}
    # the scatter and both consume kernels share class names with bench.py's timers
    for k, a in agg.items():
        n = max(a["n"], 1)
        res["kernels"][k] = {"launches": a["n"], "bytes_per_launch": (a["fetch"] + a["write"]) / n,
                             "read_bytes_per_launch": a["fetch"] / n, "write_bytes_per_launch": a["write"] / n}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
