"""Host-side view of the idle GPU gaps of one broadcast step (development aid): for each gap above
a threshold between two kernels of a rocprofv3 kernel trace, the HIP API calls the host made
meanwhile (from the same run's --hip-trace).

    rocprofv3 --kernel-trace --hip-trace --output-format csv -d <dir> -o c4 -- python3 bench.py ...
    python3 tools/api_gaps.py <dir> [step index] [min gap us] [max gaps shown]
"""
import csv
import glob
import os
import sys


def load(d, name):
    p = glob.glob(os.path.join(d, "**", f"*{name}.csv"), recursive=True)[0]
    with open(p) as f:
        return list(csv.DictReader(f))


def short(n):
    for p in ("void ", "p2pg::", "(anonymous namespace)::"):
        n = n.replace(p, "")
    return n.split("(")[0][:34]


def main():
    d = sys.argv[1]
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    thr = float(sys.argv[3]) if len(sys.argv) > 3 else 15.0
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in load(d, "kernel_trace"))
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
                 for r in load(d, "hip_api_trace"))
    seeds = [i for i, k in enumerate(ks) if "k_seed" in k[2]]
    a, b = seeds[step], (seeds[step + 1] if step + 1 < len(seeds) else len(ks))
    gaps = []
    tot = {}
    for i in range(a + 1, b):
        g = ks[i][0] - ks[i - 1][1]
        if g > thr * 1e3:
            gaps.append((g, i))
            t0, t1 = ks[i - 1][1], ks[i][0]
            for x in api:
                if x[1] > t0 and x[0] < t1:
                    ov = min(x[1], t1) - max(x[0], t0)
                    tot[x[2]] = tot.get(x[2], 0) + ov
    print(f"step {step}: {len(gaps)} gaps > {thr} us, {sum(g for g, _ in gaps) / 1e3:.1f} us in all")
    print("API time inside those gaps (us):",
          {k: round(v / 1e3, 1) for k, v in sorted(tot.items(), key=lambda x: -x[1])})
    for g, i in sorted(gaps, reverse=True)[:top]:
        t0, t1 = ks[i - 1][1], ks[i][0]
        print(f"--- {g / 1e3:.1f} us: {short(ks[i - 1][2])} -> {short(ks[i][2])}")
        for x in api:
            if x[1] > t0 - 2000 and x[0] < t1:
                print(f"   {(x[0] - t0) / 1e3:8.1f} .. {(x[1] - t0) / 1e3:8.1f}  {x[2]}")


if __name__ == "__main__":
    main()
