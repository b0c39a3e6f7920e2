#!/usr/bin/env python3
"""Copy the judged evidence of a GPU session from gpurun_out/ into profiles/ (tracked):
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (gpurun_out/prof)
  profiles/<tag>_bench.json         the bench.py JSON line (gpurun_out/bench.log)
  profiles/<tag>_pmc_canonical.json PMC averages of the step kernel + HBM bytes per launch
usage: python scripts/save_profiles.py <tag> [pmc_tag]"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
pmc_tag = sys.argv[2] if len(sys.argv) > 2 else "pmc"
out = os.path.join(ROOT, "profiles")
os.makedirs(out, exist_ok=True)
g = os.path.join(ROOT, "gpurun_out")

stats = os.path.join(g, "prof", "run_kernel_stats.csv")
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(out, f"{tag}_kernel_stats.csv"))
    for r in csv.DictReader(open(stats)):
        if "walker_step" in r["Name"]:
            print(f"rocprof: {r['Name'][:80]}  calls {r['Calls']}  avg {float(r['AverageNs']) / 1e3:.2f} us")
stats1 = os.path.join(g, "prof_l1", "run_kernel_stats.csv")   # one full-batch launch per step (lanes 1)
if os.path.exists(stats1):
    shutil.copy(stats1, os.path.join(out, f"{tag}_kernel_stats_lanes1.csv"))
span = os.path.join(g, "trace_span.log")
if os.path.exists(span):
    lines = [l for l in open(span) if l.startswith("{")]
    if lines:
        open(os.path.join(out, f"{tag}_trace_span.json"), "w").write(lines[-1])
for extra in ("lanes1", "balance", "ragged"):
    f = os.path.join(g, f"bench_{extra}.log")
    if os.path.exists(f):
        lines = [l for l in open(f) if l.startswith("{")]
        if lines:
            open(os.path.join(out, f"{tag}_bench_{extra}.json"), "w").write(lines[-1])
bench = os.path.join(g, "bench.log")
if os.path.exists(bench):
    lines = [l for l in open(bench) if l.startswith("{")]
    if lines:
        open(os.path.join(out, f"{tag}_bench.json"), "w").write(lines[-1])
        d = json.loads(lines[-1])
        print(f"bench: {d['value']:.4g} {d['unit']}  {d['ms_per_step'] * 1e3:.2f} us/step  frac {d['roofline']['frac']}")
summ = os.path.join(g, f"{pmc_tag}_summary.json")
if os.path.exists(summ):
    c = json.load(open(summ))
    hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    json.dump({"workload": "canonical", "walkers": 65536, "kernel": "walker_step_lean<true,3,false,false> (default uniform path)",
               "source": "rocprofv3 --pmc, 6 separate passes over scripts/prof_run.py (65536 canonical walkers, "
                         "30 steps), per-dispatch averages (scripts/gpu_pmc.sh, scripts/pmc_summary.py)",
               "hbm_bytes_per_launch": round(hbm),
               "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024  (gfx950: FETCH_SIZE reports half of wide streaming "
                          "reads; MI355X_MICROARCH.md HBM section)",
               "algorithmic_bytes_per_launch": 2440 * 65536, "counters": c},
              open(os.path.join(out, f"{tag}_pmc_canonical.json"), "w"), indent=1)
    print(f"pmc: {hbm:.4g} HBM bytes/launch")
