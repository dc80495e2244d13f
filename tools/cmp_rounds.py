"""Compare per-round kernel times of round_profile.py outputs (development aid).
    python tools/cmp_rounds.py gpurun_out/rounds_c4.json gpurun_out/rounds_c4_g8.json ..."""
import json
import sys


def load(p):
    d = json.load(open(p))
    run = d["runs"][-1]
    return run.get("wall_ms"), run["rounds"]


def main():
    files = sys.argv[1:]
    data = [load(f) for f in files]
    print("wall_ms", [round(w or 0, 1) for w, _ in data])
    tot = [{} for _ in files]
    n = max(len(r) for _, r in data)
    for i in range(n):
        row = []
        for k, (_, r) in enumerate(data):
            if i < len(r):
                km = r[i]["kernel_ms"]
                for c, v in km.items():
                    tot[k][c] = tot[k].get(c, 0) + v
                row.append(" ".join(f"{c[:9]}={v:.2f}" for c, v in km.items() if v > 0.05))
        if any(row):
            print(i, " | ".join(row))
    for k, f in enumerate(files):
        print(f, {c: round(v, 1) for c, v in tot[k].items() if v})


if __name__ == "__main__":
    main()
