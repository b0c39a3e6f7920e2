#!/usr/bin/env python3
"""In-process A/B of the lean step-kernel variants on the canonical 65,536-walker batch: interleaved rounds
in ONE process (cdna_hip_programming.md §5.4 rule 24).  libwalker_hip.so re-reads the WG_LEAN_* knobs on
every wg_step call.   usage: python scripts/lean_ab.py [rounds] [variant ...]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402
from walker_gym_amd.synthetic import canonical_walkers  # noqa: E402

VARIANTS = {
    "lean": {},
    "persist": {"WG_LEAN_PERSIST": "1"},
    "pf": {"WG_LEAN_PERSIST": "2"},
    "quo": {"WG_LEAN_QUO": "1"},
    "quo_w2": {"WG_LEAN_QUO": "1", "WG_LEAN_WAVES": "2"},
    "quo_w1": {"WG_LEAN_QUO": "1", "WG_LEAN_WAVES": "1"},
    "quo_pf": {"WG_LEAN_QUO": "1", "WG_LEAN_PERSIST": "2"},
    "lean_w2": {"WG_LEAN_WAVES": "2"},
    "lean_w1": {"WG_LEAN_WAVES": "1"},
    "L1": {"WG_LANES": "1"},
    "split40": {"WG_LANES_SPLIT": "0.4"},
    "split30": {"WG_LANES_SPLIT": "0.3"},
    "split60": {"WG_LANES_SPLIT": "0.6"},
    "sprio_hi": {"WG_LANES_PRIO": "-1"},
    "sprio_hi_L3": {"WG_LANES_PRIO": "-1", "WG_LANES": "3"},
    "prio0": {"WG_LEAN_PRIO": "0"},
    "prio1": {"WG_LEAN_PRIO": "1"},
    "prio2": {"WG_LEAN_PRIO": "2"},
    "prio1_L1": {"WG_LEAN_PRIO": "1", "WG_LANES": "1"},
    "prio2_L1": {"WG_LEAN_PRIO": "2", "WG_LANES": "1"},
    "L3": {"WG_LANES": "3"},
    "w2_L3": {"WG_LEAN_WAVES": "2", "WG_LANES": "3"},
    "w1_L4": {"WG_LEAN_WAVES": "1", "WG_LANES": "4"},
}
KEYS = ("WG_LEAN_PERSIST", "WG_LEAN_QUO", "WG_LEAN_WAVES", "WG_LEAN_PER_CU", "WG_LEAN_BLOCKS", "WG_LANES", "WG_LEAN_PRIO", "WG_LANES_PRIO", "WG_LANES_SPLIT")


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    names = sys.argv[2:] or list(VARIANTS)
    n, steps = 65536, 100
    env = BatchedPhysicsEnv(canonical_walkers(n, seed=0), in3d=1)
    acts = (torch.rand((steps, n, 8), device="cuda") * 2 - 1).contiguous()
    warm = acts[:10].contiguous()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {k: [] for k in names}
    geo = {}
    for r in range(rounds):
        for name in names:
            for k in KEYS:
                os.environ.pop(k, None)
            os.environ.update(VARIANTS[name])
            env.run(warm, 10)
            e0.record()
            env.run(acts, steps)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / steps * 1e3)
            geo[name] = env.launch_geometry()
        print(f"round {r}: " + "  ".join(f"{k} {v[-1]:.1f}" for k, v in res.items()), flush=True)
    for k, v in res.items():
        print(f"{k:8s} median {statistics.median(v):6.1f} us  min {min(v):6.1f} us  {geo[k]}", flush=True)


if __name__ == "__main__":
    main()
