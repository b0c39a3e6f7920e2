#!/usr/bin/env python3
"""Copy the judged pieces of a GPU session from gpurun_out/ (scratch) into profiles/ (tracked):
bench JSON lines (<name>.log -> profiles/<name>.json), rocprofv3 --stats summaries (<name>/run_kernel_stats.csv ->
profiles/<name>_kernel_stats.csv) with a per-grid summary of the trace (profiles/<name>_kernel_groups.json), and
PMC summaries (<name>_summary.json -> profiles/<name>.json).   usage: keep_profiles.py <prefix>..."""
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G, P = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles")
for pre in sys.argv[1:]:
    for log in sorted(glob.glob(os.path.join(G, pre + "*.log"))):
        name = os.path.basename(log)[:-4]
        lines = [l for l in open(log, errors="replace") if l.startswith("{\"metric\"")]
        if lines:
            open(os.path.join(P, name + ".json"), "w").write(json.dumps(json.loads(lines[-1]), indent=1) + "\n")
            print("bench", name)
    for d in sorted(glob.glob(os.path.join(G, pre + "*/run_kernel_stats.csv"))):
        name = os.path.basename(os.path.dirname(d))
        shutil.copy(d, os.path.join(P, name + "_kernel_stats.csv"))
        tr = os.path.join(os.path.dirname(d), "run_kernel_trace.csv")
        # launches 200..399 of each grid: the bench's timed single-launch control (trace_kernels.py)
        subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "trace_kernels.py"), tr, "200",
                        os.path.join(P, name + "_kernel_groups.json"), "200"], check=True, capture_output=True)
        print("rocprof", name)
    for s in sorted(glob.glob(os.path.join(G, pre + "*_summary.json"))):
        name = os.path.basename(s)[:-len("_summary.json")]
        shutil.copy(s, os.path.join(P, name + ".json"))
        print("pmc", name)
