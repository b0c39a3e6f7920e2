#!/usr/bin/env python3
"""Step-kernel durations from a rocprofv3 --kernel-trace CSV, grouped by (kernel, grid size): a full-batch launch
(bench.py's single-launch control, or `--lanes 1`) and the half-batch launches of 2 walker ranges have different
grids, which the --stats summary averages together.  The last `tail` launches of each group are the timed ones, or,
with `skip`, launches skip .. skip + tail - 1 of each group (bench.py's full-grid launches run in the order: 200 warm-up
control launches, the 200 timed control launches, then the closed-loop step() and policy loops, so `200 200` selects
the control launches that `roofline.kernel_ms_per_launch` times with events).

    python scripts/trace_kernels.py <run_kernel_trace.csv> [tail] [out.json] [skip]"""
import csv
import json
import statistics
import sys

path = sys.argv[1]
tail = int(sys.argv[2]) if len(sys.argv) > 2 else 0
skip = int(sys.argv[4]) if len(sys.argv) > 4 else None
groups = {}
for r in csv.DictReader(open(path)):
    if "walker_step" not in r["Kernel_Name"]:
        continue
    name = r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0]
    key = (name, int(r["Grid_Size_X"]))
    groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = []
for (name, grid), d in sorted(groups.items()):
    t = (d[skip:skip + tail] if skip is not None and len(d) >= skip + tail else d[-tail:]) if tail else d
    out.append({"kernel": name, "grid_threads": grid, "launches": len(d), "timed": len(t),
                "window": (f"launches {skip}..{skip + tail - 1}" if skip is not None and tail and len(d) >= skip + tail
                           else f"last {len(t)}"),
                "avg_us": round(sum(t) / len(t), 3), "median_us": round(statistics.median(t), 3),
                "min_us": round(min(t), 3), "max_us": round(max(t), 3)})
for o in out:
    print(json.dumps(o))
if len(sys.argv) > 3:
    json.dump({"source": path, "groups": out}, open(sys.argv[3], "w"), indent=1)
