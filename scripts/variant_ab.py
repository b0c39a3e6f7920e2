#!/usr/bin/env python3
"""Compile-time A/B of the step kernel (profiling aid, not product).

    python scripts/variant_ab.py build NAME=FLAGS ...     # here (CPU): ab_session/lib_NAME.so, e.g.
                                                          #   base= abl1=-DWG_ABLATE=1 (a variant is any -D flag)
    python scripts/variant_ab.py run [rounds] [workload] [NAME:ENV=V,ENV=V ...]
                                                          # GPU box: every .so in ab_session/ plus env variants of the
                                                          # in-tree library, interleaved rounds

Each (variant, round) runs in its own process (WALKER_HIP_LIB picks the library) on the bench workload and
reports the per-launch time with HIP events for one full-batch launch per step (lanes 1) and for bench.py's
default walker ranges (lanes 2); the summary is the median over rounds.  WG_AB_RESIDENT=1 times run(resident=True)
(one wg_rollout launch for all steps) instead.  Results are written to
gpurun_out/variant_ab.json."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "ab_session")   # git-ignored; emptied after each A/B session


def build(specs):
    from walker_gym_amd import build as wb
    os.makedirs(OUT, exist_ok=True)
    jobs = []
    for spec in specs:
        name, _, flags = spec.partition("=")
        cmd = wb.command(os.path.join(OUT, f"lib_{name}.so"))
        cmd = cmd[:-1] + flags.split() + cmd[-1:]
        jobs.append((name, subprocess.Popen(cmd)))
    for name, j in jobs:
        assert j.wait() == 0, name
        print("built", name)


def time_one(lib, workload, steps=200, warm=20):
    os.environ["WALKER_HIP_LIB"] = lib
    import torch
    from bench import make_spec
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    n = int(os.environ.get("WG_N", "65536"))
    spec, params = make_spec(workload, n, seed=1000)
    env = BatchedPhysicsEnv(spec, device="cuda:0", **params)
    acts = (torch.rand((steps, n, env.batch.A), device="cuda:0") * 2 - 1).contiguous()
    res = {}
    resident = os.environ.get("WG_AB_RESIDENT", "0") == "1"   # time run(resident=True): one launch for all steps
    for lanes in (1, 2):
        env.run(acts[:warm].contiguous(), warm, lanes=lanes, resident=resident)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.run(acts, steps, lanes=lanes, resident=resident)
        e1.record()
        torch.cuda.synchronize()
        res[f"lanes{lanes}"] = e0.elapsed_time(e1) / steps * 1e3
    return res


def run(rounds, workload, env_specs=()):
    variants = [(f[4:-3], os.path.join(OUT, f), {}) for f in sorted(os.listdir(OUT)) if f.endswith(".so")] \
        if os.path.isdir(OUT) else []
    only = [x for x in os.environ.get("WG_AB_ONLY", "").split(",") if x]   # a subset of the libraries by name
    if only:
        variants = [v for v in variants if v[0] in only]
    lib = os.path.join(ROOT, "walker_gym_amd", "libwalker_hip.so")
    for spec in env_specs:
        name, _, kv = spec.partition(":")
        variants.append((name, lib, dict(x.split("=", 1) for x in kv.split(",") if x)))
    allr = {name: [] for name, _, _ in variants}
    for r in range(rounds):
        for name, path, env in variants:
            p = subprocess.run([sys.executable, __file__, "one", path, workload], capture_output=True,
                               text=True, timeout=300, env=dict(os.environ, **env))
            if p.returncode:
                print(name, "FAILED", p.stderr[-400:], flush=True)
                raise SystemExit(1)
            allr[name].append(json.loads(p.stdout.strip().splitlines()[-1]))
            print(r, name, p.stdout.strip().splitlines()[-1], flush=True)
    summ = {k: {m: round(statistics.median(x[m] for x in v), 2) for m in v[0]} for k, v in allr.items()}
    for k, v in summ.items():
        print(f"{k:16s} " + "  ".join(f"{m} {x:7.2f} us" for m, x in v.items()))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump({"workload": workload, "rounds": rounds, "median_us_per_step": summ, "all": allr},
              open(os.path.join(ROOT, "gpurun_out", f"variant_ab_{workload}.json"), "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    elif sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 5, sys.argv[3] if len(sys.argv) > 3 else "canonical",
            sys.argv[4:])
    else:
        print(json.dumps(time_one(sys.argv[2], sys.argv[3])))
