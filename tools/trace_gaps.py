"""Idle time between kernels, per broadcast step, from a rocprofv3 kernel trace (development aid).

    rocprofv3 --kernel-trace --output-format csv -d <dir> -o c4 -- python3 bench.py --steps 3 ...
    python3 tools/trace_gaps.py <dir>/.../c4_kernel_trace.csv [top]

A step is cut at each k_seed dispatch (round 0), from the end of the fill that precedes it (the
reset's memsets) to the last kernel before the next fill.  Prints per step: device span, busy time
(union of kernel intervals), idle time, and the largest gaps with the kernels on either side."""
import csv
import glob
import os
import sys


def load(path):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    with open(path) as f:
        rows = list(csv.DictReader(f))
    out = []
    for r in rows:
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    out.sort()
    return out


def short(name):
    for p in ("void ", "p2pg::", "(anonymous namespace)::"):
        name = name.replace(p, "")
    return name.split("(")[0][:60]


def main():
    ks = load(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    seeds = [i for i, k in enumerate(ks) if "k_seed" in k[2]]
    for si, s in enumerate(seeds):
        # back up over the reset's fills / row zeroing that precede the seed
        a = s
        while a > 0 and ("fill" in ks[a - 1][2].lower() or "zero_rows" in ks[a - 1][2]):
            a -= 1
        b = seeds[si + 1] if si + 1 < len(seeds) else len(ks)
        while b - 1 > s and ("fill" in ks[b - 1][2].lower() or "zero_rows" in ks[b - 1][2]):
            b -= 1
        seg = ks[a:b]
        t0, t1 = seg[0][0], max(k[1] for k in seg)
        busy, cur_s, cur_e = 0, seg[0][0], seg[0][1]
        gaps = []
        for i in range(1, len(seg)):
            st, en, nm = seg[i]
            if st > cur_e:
                busy += cur_e - cur_s
                gaps.append((st - cur_e, short(seg[i - 1][2]), short(nm)))
                cur_s, cur_e = st, en
            else:
                cur_e = max(cur_e, en)
        busy += cur_e - cur_s
        span = (t1 - t0) / 1e6
        print(f"step {si}: {len(seg)} kernels, span {span:.3f} ms, busy {busy / 1e6:.3f} ms, "
              f"idle {span - busy / 1e6:.3f} ms in {len(gaps)} gaps; fills before seed: {s - a}")
        gaps.sort(reverse=True)
        for g, x, y in gaps[:top]:
            print(f"   {g / 1e3:8.1f} us  {x}  ->  {y}")
        by = {}
        for st, en, nm in seg:
            k = short(nm)
            t, n = by.get(k, (0, 0))
            by[k] = (t + en - st, n + 1)
        for k, (t, n) in sorted(by.items(), key=lambda x: -x[1][0])[:top]:
            print(f"   busy {t / 1e6:8.3f} ms in {n:4d}  {k}")


if __name__ == "__main__":
    main()
