"""Per-dispatch SQ issue/stall breakdown of one kernel from rocprofv3 PMC passes
(tools/pmc_passes.sh run with SQ counter groups; MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY
+ ACTIVE_INST_ANY = WAVE_CYCLES, all in quad-cycles).

    python tools/pmc_sq_report.py gpurun_out/pmc_sq k_gossip_fused
"""
import sys

from pmc_report import load


def main():
    d, key = sys.argv[1], sys.argv[2]
    disp = load(d)
    ids = sorted(i for i in disp if key in disp[i]["name"])
    ids = ids[len(ids) // 2:]  # the measured broadcast
    tot = {"ns": 0}
    print(f"{'ms':>7s} {'wait%':>6s} {'issue%':>6s} {'activ%':>6s} {'valu%':>6s} {'lds%':>5s} {'vmem%':>6s} "
          f"{'VALU/wv':>8s} {'VMrd/wv':>8s} {'VMwr/wv':>8s} {'LDS/wv':>7s} {'bankc%':>6s} {'waves':>8s}")
    for i in ids:
        e = disp[i]
        for c, v in e.items():
            if isinstance(v, (int, float)):
                tot[c] = tot.get(c, 0) + v
        row(e)
    print("total:")
    row(tot)


def row(e):
    wc = max(e.get("SQ_WAVE_CYCLES", 0), 1)
    waves = max(e.get("SQ_WAVES", 0), 1)
    print(f"{e['ns'] / 1e6:7.2f} {100 * e.get('SQ_WAIT_ANY', 0) / wc:6.1f} "
          f"{100 * e.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} {100 * e.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.1f} "
          f"{100 * e.get('SQ_ACTIVE_INST_VALU', 0) / wc:6.1f} {100 * e.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.1f} "
          f"{100 * e.get('SQ_ACTIVE_INST_VMEM', 0) / wc:6.1f} "
          f"{e.get('SQ_INSTS_VALU', 0) / waves:8.0f} {e.get('SQ_INSTS_VMEM_RD', 0) / waves:8.0f} "
          f"{e.get('SQ_INSTS_VMEM_WR', 0) / waves:8.0f} {e.get('SQ_INSTS_LDS', 0) / waves:7.0f} "
          f"{100 * e.get('SQ_LDS_BANK_CONFLICT', 0) / max(e.get('SQ_LDS_IDX_ACTIVE', 0), 1):6.1f} "
          f"{waves:8.0f}")


if __name__ == "__main__":
    main()
