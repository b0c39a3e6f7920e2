#!/usr/bin/env python3
"""Step-kernel durations from a rocprofv3 --kernel-trace CSV, grouped by (kernel, grid size): a full-batch launch
(bench.py's single-launch control, or `--lanes 1`) and the half-batch launches of 2 walker ranges have different
grids, which the --stats summary averages together.  The last `tail` launches of each group are the timed ones, or,
with `skip`, launches skip .. skip + tail - 1 of each group (bench.py's full-grid launches run in the order: 200 warm-up
control launches, the 200 timed control launches, then the closed-loop step() and policy loops, so `200 200` selects
the control launches that `roofline.kernel_ms_per_launch` times with events).

    python scripts/trace_kernels.py <run_kernel_trace.csv> [tail] [out.json] [skip]

Window mode: the per-step time of a multi-range region from the launch timestamps themselves —
launches skip .. skip + count - 1 of the step kernel with `grid` threads (bench.py's timed region of K steps over 2
walker ranges is the half-grid launches 2W .. 2W + 2K - 1 after its W warm-up steps), their span (first start to last
end) divided by `steps`, the launch spacing and duration per hardware queue, and how much of the span both ranges
were running at once:

    python scripts/trace_kernels.py <run_kernel_trace.csv> --window GRID SKIP COUNT STEPS [out.json [key=value ...]]

(GRID 0: every step launch whose grid is not the largest one — the walker ranges of a ragged batch have grids of their
own sizes.)

(key=value pairs are stored in the JSON: bench.py picks a window record up by its `workload` and `walkers`.)"""
import csv
import json
import statistics
import sys


def launches(path):
    for r in csv.DictReader(open(path)):
        if "walker_step" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0]
        yield name, int(r["Grid_Size_X"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?")


def window(path, grid, skip, count, steps):
    allw = list(launches(path))
    if grid == 0:   # the walker-range launches: every grid but the largest (the full-batch control launches)
        big = max(x[1] for x in allw)
        w = [x for x in allw if x[1] != big][skip:skip + count]
    else:
        w = [x for x in allw if x[1] == grid][skip:skip + count]
    if len(w) < count:
        raise SystemExit(f"only {len(w)} launches of grid {grid} after skipping {skip}")
    t0, t1 = min(x[2] for x in w), max(x[3] for x in w)
    per_q = {}
    for x in w:
        per_q.setdefault(x[4], []).append((x[2], x[3]))
    queues = []
    for q, v in sorted(per_q.items()):
        v.sort()
        gaps = [(b[0] - a[0]) / 1e3 for a, b in zip(v, v[1:])]
        queues.append({"queue": q, "launches": len(v), "avg_spacing_us": round(sum(gaps) / max(1, len(gaps)), 3),
                       "avg_duration_us": round(sum(b - a for a, b in v) / len(v) / 1e3, 3)})
    ev = sorted([(x[2], 1) for x in w] + [(x[3], -1) for x in w])
    busy = {0: 0, 1: 0, 2: 0}
    cur, last = 0, None
    for t, d in ev:
        if last is not None:
            busy[min(cur, 2)] += t - last
        cur, last = cur + d, t
    span = t1 - t0
    return {"kernel": w[0][0], "grid_threads": grid if grid else sorted({x[1] for x in w}), "launches": count, "window": f"launches {skip}..{skip + count - 1}",
            "steps": steps, "span_us": round(span / 1e3, 3), "us_per_step": round(span / 1e3 / steps, 4),
            "queues": queues, "share_two_or_more_running": round(busy[2] / span, 4),
            "share_one_running": round(busy[1] / span, 4), "share_idle": round(busy[0] / span, 4)}


def groups(path, tail, skip):
    g = {}
    for name, grid, s, e, _ in launches(path):
        g.setdefault((name, grid), []).append((e - s) / 1e3)
    out = []
    for (name, grid), d in sorted(g.items()):
        t = (d[skip:skip + tail] if skip is not None and len(d) >= skip + tail else d[-tail:]) if tail else d
        out.append({"kernel": name, "grid_threads": grid, "launches": len(d), "timed": len(t),
                    "window": (f"launches {skip}..{skip + tail - 1}" if skip is not None and tail and len(d) >= skip + tail
                               else f"last {len(t)}"),
                    "avg_us": round(sum(t) / len(t), 3), "median_us": round(statistics.median(t), 3),
                    "min_us": round(min(t), 3), "max_us": round(max(t), 3)})
    return out


if __name__ == "__main__":
    path = sys.argv[1]
    if len(sys.argv) > 2 and sys.argv[2] == "--window":
        grid, skip, count, steps = (int(x) for x in sys.argv[3:7])
        res = dict(window(path, grid, skip, count, steps), source=path)
        for kv in sys.argv[8:]:
            k, _, v = kv.partition("=")
            res[k] = int(v) if v.isdigit() else v
        print(json.dumps(res))
        if len(sys.argv) > 7:
            json.dump(res, open(sys.argv[7], "w"), indent=1)
        sys.exit(0)
    tail = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else None
    out = groups(path, tail, skip)
    for o in out:
        print(json.dumps(o))
    if len(sys.argv) > 3:
        json.dump({"source": path, "groups": out}, open(sys.argv[3], "w"), indent=1)
