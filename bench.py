#!/usr/bin/env python3
"""Headline benchmark: env-steps/sec of the batched walker stepper (BASELINE.json `metric`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--walkers 65536] [--workload canonical]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one env step (act -> springs -> env forces -> run1 -> obs/reward/done/info) over the rank's
batch, with obs/reward/done/info materialised every step.  The batch is split into 2 contiguous walker
ranges stepped on 2 HIP streams (BatchedPhysicsEnv.run lanes), one launch per range per step: every walker
takes every step, and one range's next step fills the GPU while the other's drains.  Inputs (state, topology
and a distinct U(-1,1) action tensor for every timed step) are resident in HBM before timing starts.
Weak scaling: each rank owns its own `--walkers` walkers (no data-path collective); at rollout end the
final observations are gathered with one RCCL all_gather_into_tensor (inside the timed region).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node) at 65 536 walkers; 1/2/4/8 MI355X scaling"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--walkers", type=int, default=65536, help="walkers per GPU")
    ap.add_argument("--workload", default="canonical", choices=["canonical", "balance", "ragged"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-control", action="store_true", help="skip the single-launch (lanes 1) control timing")
    return ap.parse_args()


def make_spec(workload: str, n: int, seed: int):
    from walker_gym_amd.synthetic import canonical_walkers, ragged_walkers
    from walker_gym_amd.walker import balance_spec
    if workload == "canonical":
        return canonical_walkers(n, seed=seed), dict(in3d=1)
    if workload == "balance":
        return balance_spec(n), dict(in3d=0)
    return ragged_walkers(n, seed=seed, mmin=4, mmax=32), dict(in3d=1)


def cpu_baseline(spec_fn, params, A, budget_s: float):
    """The C oracle (oracle/walker_oracle.c, the restated reference loop) on host cores, on a bounded
    sample of the same workload: single thread, then all usable cores (OpenMP over walkers)."""
    from oracle.oracle import Oracle
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    n = 4096
    spec = spec_fn(n)
    rng = np.random.default_rng(123)
    acts = rng.uniform(-1, 1, (8, n, A)).astype(np.float32)
    res = {}
    for label, thr in (("1", 1), ("all", cores)):
        orc = Oracle(spec, params, n_threads=thr)
        t0 = time.perf_counter(); orc.step(acts[0]); probe = time.perf_counter() - t0
        share = budget_s * (0.3 if thr == 1 else 0.7)
        steps = int(max(2, min(2000, share / max(probe, 1e-6))))
        t0 = time.perf_counter()
        for s in range(steps):
            orc.step(acts[s % 8])
        dt = time.perf_counter() - t0
        res[label] = (n * steps / dt, steps, thr)
    v_all, steps_all, thr_all = res["all"]
    return {"value": round(v_all, 1), "unit": "env-steps/s", "cores": thr_all, "kind": "port",
            "sample": f"{n} walkers x {steps_all} steps of the same workload (C oracle restating "
                      f"gym/engine.py + gym/optimized_env.py), OpenMP over walkers",
            "value_1core": round(res["1"][0], 1), "sample_1core": f"{n} walkers x {res['1'][1]} steps, 1 thread"}


def load_traffic(workload: str, walkers: int):
    """HBM bytes per launch from a committed rocprofv3 PMC run (profiles/*pmc*.json), if present."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), key=os.path.getmtime):   # newest last
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("workload") == workload and d.get("walkers") == walkers and "hbm_bytes_per_launch" in d:
            best = d
    return best


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.layout import algorithmic_bytes_per_walker_step, layout_bytes_per_walker_step

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("WG_DIST_BACKEND", "nccl")   # nccl = RCCL; gloo only to rehearse ranks on one GPU
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    N = args.walkers
    spec, params = make_spec(args.workload, N, seed=1000 + rank)
    env = BatchedPhysicsEnv(spec, device=dev, **params)
    A = env.batch.A
    M, K = env.batch.M, env.batch.K
    gen = torch.Generator(device=dev)
    gen.manual_seed(7 + rank)
    acts_w = (torch.rand((max(args.warmup, 1), N, A), generator=gen, device=dev) * 2 - 1).contiguous()
    acts = (torch.rand((args.steps, N, A), generator=gen, device=dev) * 2 - 1).contiguous()
    gather_buf = torch.empty((world * N, env.obs_dim), dtype=torch.float32, device=dev) if world > 1 else None

    # warmup (untimed)
    if args.warmup > 0:
        env.run(acts_w, args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    env.run(acts, args.steps)
    ev1.record(stream)
    if world > 1 and not args.no_gather:
        if backend == "nccl":
            dist.all_gather_into_tensor(gather_buf, env.obs)  # rollout-end observation gather (RCCL)
        else:
            dist.all_gather(list(gather_buf.chunk(world, 0)), env.obs)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps              # stream-ordered, per launch

    wall_t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(wall_t, op=dist.ReduceOp.MAX)
    wall_max = float(wall_t.item())

    lanes = env._lanes(None)
    single_ms = None
    if rank == 0 and lanes > 1 and not args.no_control:
        # control: the same kernel as one full-batch launch per step (lanes 1), events on its stream.  This is
        # the per-dispatch duration a rocprofv3 kernel trace reports (tracing serialises the two streams).
        n1 = max(20, min(args.steps, 100))
        env.run(acts[:n1], n1, lanes=1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        env.run(acts[:n1], n1, lanes=1)
        e1.record(stream)
        torch.cuda.synchronize()
        single_ms = e0.elapsed_time(e1) / n1

    if rank == 0:
        D = env.obs_dim
        B = algorithmic_bytes_per_walker_step(M, K, A, D)
        B_layout = layout_bytes_per_walker_step(M, K, A, D)
        achieved = B * N / (step_ms * 1e-3) / 1e9
        tr = load_traffic(args.workload, N)
        geo = env.launch_geometry()
        line = {
            "metric": METRIC,
            "value": round(world * N * args.steps / wall_max, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max * 1e3 / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded; SURVEY §8(d) canonical walker; U(-1,1) actions, distinct per step)",
            "config": {"workload": f"{args.workload} walkers, {N} per GPU (M={M}, K={K}, A={A}, obs D={D}), "
                                   "one fused act+physics+observe launch per env step per walker range "
                                   f"({env._lanes(None)} ranges on {env._lanes(None)} streams)",
                       "walkers_per_gpu": N, "total_walkers": world * N, "M": M, "K": K, "A": A, "obs_dim": D,
                       "parallelism": f"dp{world}", "rollout_gather": world > 1 and not args.no_gather,
                       "lanes": env._lanes(None), "launch": geo},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": (tr["hbm_bytes_per_launch"] if tr else None),
                         "bytes_per_walker_step": B, "layout_bytes_per_walker_step": B_layout,
                         "kernel_ms_per_step_events": round(step_ms, 5),
                         "note": (f"achieved = N*B / event time per step; a step is {lanes} concurrent launches "
                                  "(one per walker range)" if lanes > 1 else "achieved = N*B / event time per launch")},
        }
        if single_ms:
            a1 = B * N / (single_ms * 1e-3) / 1e9
            line["roofline"]["single_launch"] = {"lanes": 1, "kernel_ms_per_launch_events": round(single_ms, 5),
                                                 "achieved": round(a1, 1), "frac": round(a1 / HBM_PEAK_GBS, 4)}
        if world == 1 and not args.no_cpu_baseline:
            fn = lambda n: make_spec(args.workload, n, seed=99)[0]
            line["cpu_baseline"] = cpu_baseline(fn, params, A, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
