"""Per-launch durations (us) of the sparse-round kernels in a rocprofv3 kernel trace of
tools/round_profile.py (one c4 broadcast): python3 tools/sparse_trace_report.py <trace dir>"""
import csv
import glob
import sys

KEYS = ("k_sparse_words<false>", "k_chunk_scan", "k_sparse_words<true>", "k_sparse_push",
        "k_touched_bits", "k_gossip_update1", "k_pull1", "k_gossip_scatter", "k_wide_zero",
        "k_wide_push", "k_gossip_fused")
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
per = {k: [] for k in KEYS}
for r in rows:
    for k in KEYS:
        if k in r["Kernel_Name"]:
            per[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            break
for k, v in per.items():
    if v:
        print(f"{k:24s} n={len(v):3d} sum={sum(v) / 1e3:7.2f} ms  first 30: {[round(x) for x in v[:30]]}")
