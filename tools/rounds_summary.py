"""Print a per-round table (stats + kernel ms) of tools/round_profile.py output."""
import json
import sys

for path in sys.argv[1:]:
    d = json.load(open(path))
    run = d["runs"][-1]
    print(path, "wall %.1f ms" % run["wall_ms"])
    for r in run["rounds"]:
        km = {k: round(v, 2) for k, v in r["kernel_ms"].items() if v > 0.005}
        av = max(r["active_vertices"], 1)
        print("%2d new %9.3g av %9.3g aw/av %5.1f sc %9.3g tw %9.3g form %d %s" % (
            r["round"], r["new_deliveries"], r["active_vertices"], r["active_words"] / av,
            r["scatter_words"], r["touched_words"], r.get("push_form", 0), km))
