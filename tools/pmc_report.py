"""Merge rocprofv3 PMC passes (tools/pmc_passes.sh) by dispatch and summarise per kernel.

    python tools/pmc_report.py gpurun_out/pmc_c4 [--rounds]
HBM bytes follow MI355X_MICROARCH.md: FETCH_SIZE (KB) counts 64 B per TCC_EA0_RDREQ, which is
half the bytes of a wide coalesced stream on gfx950, so reads are reported both raw and x2."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    disp = defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(d, "pass*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = int(row["Dispatch_Id"])
            e = disp[k]
            e["name"] = row["Kernel_Name"]
            e["ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            e[row["Counter_Name"]] = e.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return disp


def short(n):
    for key in ("k_gossip_fused", "k_pull1", "k_pull", "k_gossip_update", "k_gossip_scatter", "k_record", "k_seed",
                "k_zero_rows", "fillBuffer", "copyBuffer"):
        if key in n:
            if key == "k_gossip_scatter":
                return "scatter_E" if ("true>(" in n or "ELb1EEEv" in n) else "scatter_atomic"
            if key.startswith("k_pull"):
                return key + ("_gossip" if ("true>(" in n or "ELb1EEEv" in n) else "_flood")
            return key
    return n[:30]


def main():
    d = sys.argv[1]
    disp = load(d)
    ids = sorted(disp)
    # second half = the measured broadcast
    half = ids[len(ids) // 2:]
    agg = defaultdict(lambda: defaultdict(float))
    rows = []
    for i in half:
        e = disp[i]
        k = short(e["name"])
        a = agg[k]
        a["n"] += 1
        for c, v in e.items():
            if isinstance(v, float) or isinstance(v, int):
                a[c] += v
        rows.append((k, e))
    print(f"{'kernel':18s} {'n':>4s} {'ms':>8s} {'FETCH GB':>9s} {'x2 GB':>8s} {'WRITE GB':>9s} {'rd TB/s(x2)':>11s} "
          f"{'TLBmiss%':>8s} {'L2hit%':>7s} {'VALU/VMEM':>9s} {'busy%':>6s}")
    for k, a in sorted(agg.items(), key=lambda x: -x[1]["ns"]):
        ms = a["ns"] / 1e6
        fg = a.get("FETCH_SIZE", 0) * 1024 / 1e9
        wg = a.get("WRITE_SIZE", 0) * 1024 / 1e9
        tm = a.get("TCP_UTCL1_TRANSLATION_MISS", 0)
        th = a.get("TCP_UTCL1_TRANSLATION_HIT", 0)
        hit = a.get("TCC_HIT", 0)
        miss = a.get("TCC_MISS", 0)
        valu = a.get("SQ_INSTS_VALU", 0)
        vm = a.get("SQ_INSTS_VMEM_RD", 0) + a.get("SQ_INSTS_VMEM_WR", 0)
        busy = a.get("SQ_ACTIVE_INST_ANY", 0) / max(a.get("SQ_WAVE_CYCLES", 1), 1)
        print(f"{k:18s} {int(a['n']):4d} {ms:8.2f} {fg:9.2f} {2*fg:8.2f} {wg:9.2f} {2*fg/max(ms,1e-9):11.2f} "
              f"{100*tm/max(tm+th,1):8.2f} {100*hit/max(hit+miss,1):7.2f} {valu/max(vm,1):9.2f} {100*busy:6.1f}")
    if "--rounds" in sys.argv:
        for k, e in rows:
            if k.startswith(("k_pull", "scatter", "k_gossip_update")):
                ms = e["ns"] / 1e6
                fg = e.get("FETCH_SIZE", 0) * 1024 / 1e9
                wg = e.get("WRITE_SIZE", 0) * 1024 / 1e9
                tm = e.get("TCP_UTCL1_TRANSLATION_MISS", 0)
                th = e.get("TCP_UTCL1_TRANSLATION_HIT", 0)
                print(f"  {k:18s} {ms:7.2f} ms  fetch {fg:7.2f} GB  write {wg:6.2f} GB  tlbmiss {100*tm/max(tm+th,1):5.2f}%"
                      f"  L2hit {100*e.get('TCC_HIT',0)/max(e.get('TCC_HIT',0)+e.get('TCC_MISS',0),1):5.1f}%")


if __name__ == "__main__":
    main()
