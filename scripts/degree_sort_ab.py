#!/usr/bin/env python3
"""Upper bound of VERDICT r4's "cut 1" (regroup canonical walkers across wave tiles by their largest mass degree, so a
wave's mass loop runs fewer iterations) without building the caller-order indirection: the SAME walkers stepped in
their generated order and in an order sorted by largest degree (the data itself permuted, identity rows), one env
each, interleaved in one process on one box.  The indirection could only add cost to the sorted figure.

    python scripts/degree_sort_ab.py [rounds] [steps]      # GPU box; writes gpurun_out/degree_sort_ab.json"""
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def max_degree(spec, N, M, K):
    ei = spec["ei"].reshape(N, K)
    ej = spec["ej"].reshape(N, K)
    deg = np.zeros((N, M), np.int32)
    for a in (ei, ej):
        np.add.at(deg, (np.repeat(np.arange(N), K), a.reshape(-1)), 1)
    return deg.max(axis=1), deg


def permute(spec, order, N, M, K, A):
    out = dict(spec)
    per = {"m": M, "pos": M, "vel": M, "acc": M, "ei": K, "ej": K, "rest": K, "k": K, "c": K, "flags": K,
           "n_muscles": 1, "minl": A, "maxl": A, "stride": A}
    for key, n in per.items():
        a = spec[key]
        out[key] = a.reshape((N, n) + a.shape[1:])[order].reshape(a.shape).copy()
    return out


def main():
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    N, M, K, A = 65536, 16, 40, 8
    spec = canonical_walkers(N, seed=1000)
    mx, _ = max_degree(spec, N, M, K)
    order = np.argsort(mx, kind="stable")
    # descending: the tiles with the longest mass loops first, the shortest last (longest-processing-time-first
    # order against the launch's drain)
    order_d = order[::-1].copy()
    # lpt: descending within each XCD's contiguous chunk of tiles (xcd_block gives XCD x the x-th eighth of the tiles,
    # dispatched in order), the walkers dealt round-robin so every chunk has the same degree mix
    order_l = np.concatenate([order_d[j::8] for j in range(8)])
    # lpt2: the same per XCD chunk of each of the two walker ranges (16 chunks: range r's launch gives XCD x its x-th
    # eighth), for the two-range step
    order_l2 = np.concatenate([order_d[j::16] for j in range(16)])
    sspec = permute(spec, order, N, M, K, A)
    dspec = permute(spec, order_l, N, M, K, A)
    d2spec = permute(spec, order_l2, N, M, K, A)
    wave_max = {"generated": float(mx.reshape(-1, 4).max(axis=1).mean()),
                "sorted": float(mx[order].reshape(-1, 4).max(axis=1).mean()),
                "sorted_lpt": float(mx[order_l].reshape(-1, 4).max(axis=1).mean()),
                "sorted_lpt2": float(mx[order_l2].reshape(-1, 4).max(axis=1).mean())}
    envs = {"generated": BatchedPhysicsEnv(spec, device="cuda:0", in3d=1),
            "sorted": BatchedPhysicsEnv(sspec, device="cuda:0", in3d=1),
            "sorted_lpt": BatchedPhysicsEnv(dspec, device="cuda:0", in3d=1),
            "sorted_lpt2": BatchedPhysicsEnv(d2spec, device="cuda:0", in3d=1)}
    acts = (torch.rand((steps, N, A), device="cuda:0") * 2 - 1).contiguous()
    res = {k: {"lanes1": [], "lanes2": []} for k in envs}
    for r in range(rounds):
        for name, env in envs.items():
            for lanes in (1, 2):
                env.run(acts[:20].contiguous(), 20, lanes=lanes)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                env.run(acts, steps, lanes=lanes)
                e1.record()
                torch.cuda.synchronize()
                res[name][f"lanes{lanes}"].append(round(e0.elapsed_time(e1) / steps * 1e3, 3))
        print(r, json.dumps({k: {m: v[m][-1] for m in v} for k, v in res.items()}), flush=True)
    out = {"walkers": N, "steps": steps, "rounds": rounds, "mean_wave_max_degree": wave_max,
           "median_us_per_step": {k: {m: statistics.median(v[m]) for m in v} for k, v in res.items()}, "all": res}
    print(json.dumps(out["median_us_per_step"]), json.dumps(wave_max))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "degree_sort_ab.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
