#!/usr/bin/env python3
"""Phase ablation of the step kernel (profiling aid, not product): builds libwalker_hip.so variants
with -DWG_ABLATE=<mask> (bit0 edge compute, bit1 incidence loop, bit3 reductions, bit4 obs) and times
each on the GPU in its own process.   build:  python scripts/ablate.py build   run: python scripts/ablate.py run"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build_ablate")
MASKS = [0, 1, 2, 3, 16, 19]
EXTRA = {}   # name -> extra -D flags


def build():
    from walker_gym_amd import build as wb
    os.makedirs(OUT, exist_ok=True)
    jobs = []
    variants = [(f"abl{m}", [f"-DWG_ABLATE={m}"]) for m in MASKS] + [(k, v) for k, v in EXTRA.items()]
    for name, flags in variants:
        cmd = wb.command(os.path.join(OUT, f"lib_{name}.so"))
        cmd = cmd[:-1] + flags + cmd[-1:]
        jobs.append(subprocess.Popen(cmd))
    for j in jobs:
        assert j.wait() == 0


def time_one(lib, steps=200, warm=20, n=int(os.environ.get("WG_N", "65536")), workload="canonical"):
    os.environ["WALKER_HIP_LIB"] = lib
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    env = BatchedPhysicsEnv(canonical_walkers(n, seed=0), in3d=1)
    acts = (torch.rand((steps, n, 8), device="cuda") * 2 - 1).contiguous()
    env.run(acts[:warm].contiguous(), warm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); env.run(acts, steps); e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def run():
    libs = sorted(f for f in os.listdir(OUT) if f.endswith(".so"))
    for f in libs:
        r = subprocess.run([sys.executable, __file__, "one", os.path.join(OUT, f)], capture_output=True, text=True,
                           timeout=300, env=dict(os.environ, WG_STREAM="0"))
        print(f"{f:24s} {r.stdout.strip()} {r.stderr.strip()[-200:] if r.returncode else ''}", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    elif sys.argv[1] == "run":
        run()
    else:
        print(f"{time_one(sys.argv[2]) * 1e3:.1f} us/step")
