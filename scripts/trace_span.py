#!/usr/bin/env python3
"""Per-step GPU time of the step kernels from a rocprofv3 kernel trace: the union of the step-kernel
intervals of the timed region divided by its steps (with lanes > 1 two half-batch launches overlap, so
the per-dispatch average of --stats is not the step time).  usage: trace_span.py <trace.csv> <steps> [lanes]"""
import csv
import json
import sys

path, steps = sys.argv[1], int(sys.argv[2])
lanes = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path))
               if "walker_step" in r["Kernel_Name"]))
timed = rows[-steps * lanes:]                        # the timed region's launches come last
busy, cur_s, cur_e = 0, None, None
for s, e in timed:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = timed[-1][1] - timed[0][0]
durs = [e - s for s, e in timed]
out = {"launches": len(timed), "steps": steps, "lanes": lanes, "avg_launch_ns": sum(durs) / len(durs),
       "busy_ns_per_step": busy / steps, "span_ns_per_step": span / steps}
print(json.dumps(out))
