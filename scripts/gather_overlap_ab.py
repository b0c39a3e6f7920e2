#!/usr/bin/env python3
"""Can the rollout-end gather overlap the steps without stalling them?  
Same box, world 1 under torch.distributed.run (RCCL), 65,536 canonical walkers, two walker ranges, K steps with
per-step reward / done records.  Forms, each in its own process, interleaved over rounds:
  none          the K steps alone (the reference point)
  serial        the K steps, then the gather of this rollout (obs [N, D], reward / done [K, N]): bench.py's default
  rccl          the previous rollout's gather (RCCL all_gather_into_tensor, its own stream) issued before the K steps
  rccl_ch1/2/4  the same with RCCL capped at NCCL_MAX_NCHANNELS = 1 / 2 / 4 (fewer CUs for the collective)
  rccl_hiprio   the same with the steps' streams at high priority (RCCL's stream at normal)
  copy          the previous rollout's blocks copied device-to-device into the gather buffer on a side stream (the
                copy-engine form's stand-in for a rank's own block: hipMemcpyAsync, no collective)
Reported per form: ms per step of the K steps by HIP events on the stepping stream, the wall time of the region
(steps + gather, synchronised), value (steps only) and value_incl_gather.
    python scripts/gather_overlap_ab.py [rounds=5] [K=20] [forms...]   -> gpurun_out/gather_overlap_ab.json"""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FORMS = ["none", "serial", "rccl", "rccl_ch1", "rccl_ch2", "rccl_ch4", "rccl_hiprio", "copy"]


def one(form: str, K: int) -> dict:
    import torch
    import torch.distributed as dist
    from bench import device_warm, make_spec
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.distributed import gather_rollout, gather_rollout_async
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N = int(os.environ.get("WG_N", "65536"))
    spec, params = make_spec("canonical", N, seed=1000)
    hi = form == "rccl_hiprio"
    main_st = torch.cuda.Stream(device=dev, priority=-1) if hi else torch.cuda.current_stream(dev)
    with torch.cuda.stream(main_st):
        env = BatchedPhysicsEnv(spec, device=dev, **params)
        if hi:
            env._side = [torch.cuda.Stream(device=dev, priority=-1)]
        lanes = env._lanes(None)
        env.reserve_streams(lanes)
        acts = (torch.rand((K, N, env.batch.A), device=dev) * 2 - 1).contiguous()
        env.run(acts[:1].contiguous(), 1, lanes=lanes)
        torch.cuda.synchronize()
    dist.init_process_group("nccl", device_id=dev)
    world = dist.get_world_size()
    with torch.cuda.stream(main_st):
        rec = {"reward": torch.empty((K, N), device=dev), "done": torch.empty((K, N), dtype=torch.uint8, device=dev)}
        prev = {"obs": env.obs.clone(), "reward": rec["reward"].clone(), "done": rec["done"].clone()}
        gbuf = {k: torch.empty((world * v.shape[0],) + tuple(v.shape[1:]), dtype=v.dtype, device=dev)
                for k, v in prev.items()}
        copy_st = torch.cuda.Stream(device=dev)

        def gather(src):
            return {"obs": gather_rollout(src["obs"], n_total=world * N),
                    "reward": gather_rollout(src["reward"], n_total=world * N, dim=1),
                    "done": gather_rollout(src["done"], n_total=world * N, dim=1)}
        gather(prev)                                   # RCCL's first gather of these shapes (untimed)
        torch.cuda.synchronize()
        device_warm(main_st, dev, 100)
        env.run(acts, K, lanes=lanes, record=rec)
        prep = env.prepare_run(acts, K, lanes=lanes, record=rec)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(main_st)
        pend = []
        if form.startswith("rccl"):
            pend = [gather_rollout_async(prev["obs"], n_total=world * N),
                    gather_rollout_async(prev["reward"], n_total=world * N, dim=1),
                    gather_rollout_async(prev["done"], n_total=world * N, dim=1)]
        elif form == "copy":
            copy_st.wait_stream(main_st)
            with torch.cuda.stream(copy_st):
                for k in prev:
                    gbuf[k].copy_(prev[k], non_blocking=True)
        prep()
        e1.record(main_st)
        for h in pend:
            h.wait()
        if form == "serial":
            gather({"obs": env.obs, "reward": rec["reward"], "done": rec["done"]})
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        step_ms = e0.elapsed_time(e1) / K
    dist.destroy_process_group()
    return {"form": form, "K": K, "step_ms_events": round(step_ms, 5), "wall_ms": round(wall * 1e3, 4),
            "value_steps": round(N * K / (step_ms * K * 1e-3), 1), "value_incl_gather": round(N * K / wall, 1)}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        print(json.dumps(one(sys.argv[2], int(sys.argv[3]))), flush=True)
        return
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    forms = sys.argv[3:] or FORMS
    allr = {f: [] for f in forms}
    port = 29700
    for r in range(rounds):
        for f in forms:
            env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
            if f.startswith("rccl_ch"):
                env["NCCL_MAX_NCHANNELS"] = f[len("rccl_ch"):]
            port += 1
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                   "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), "one", f, str(K)]
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
            if p.returncode:
                print(f, "FAILED", p.stderr[-600:], flush=True)
                raise SystemExit(1)
            row = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
            allr[f].append(row)
            print(r, json.dumps(row), flush=True)
    summ = {f: {m: round(statistics.median(x[m] for x in v), 5) for m in ("step_ms_events", "wall_ms", "value_steps",
                                                                            "value_incl_gather")}
            for f, v in allr.items()}
    base = summ.get("none", {}).get("step_ms_events")
    for f, v in summ.items():
        if base:
            v["step_slowdown_vs_none"] = round(v["step_ms_events"] / base - 1, 4)
        print(f"{f:12s} " + "  ".join(f"{m} {x}" for m, x in v.items()), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump({"K": K, "rounds": rounds, "median": summ, "all": allr},
              open(os.path.join(ROOT, "gpurun_out", f"gather_overlap_ab_k{K}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
