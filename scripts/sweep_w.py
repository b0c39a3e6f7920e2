#!/usr/bin/env python3
"""Walkers-per-workgroup sweep (experiment): time the canonical 65,536-walker step for several W."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one():
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    n, steps = 65536, 200
    env = BatchedPhysicsEnv(canonical_walkers(n, seed=0), in3d=1)
    acts = (torch.rand((steps, n, 8), device="cuda") * 2 - 1).contiguous()
    env.run(acts[:20].contiguous(), 20)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); env.run(acts, steps); e1.record(); torch.cuda.synchronize()
    print(f"{e0.elapsed_time(e1) / steps * 1e3:.1f} us/step  geo={env.launch_geometry()}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        one()
    else:
        for w in sys.argv[1:] or ["4", "8", "12", "16"]:
            env = dict(os.environ, WG_DEBUG_WALKERS_PER_BLOCK=w)
            r = subprocess.run([sys.executable, __file__, "one"], env=env, capture_output=True, text=True, timeout=300)
            print(f"W={w:3s} {r.stdout.strip()} {r.stderr.strip()[-300:] if r.returncode else ''}", flush=True)
