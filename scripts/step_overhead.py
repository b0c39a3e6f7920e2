#!/usr/bin/env python3
"""Closed-loop cost of BatchedPhysicsEnv.step (diagnostic, not product): host time per step() call (no sync: the
launches queue asynchronously) and the GPU time per step when the caller loops over step(), for 1 and 2 walker ranges
(step() forks and joins its ranges every step), beside the open-loop run() of the same steps.
    python scripts/step_overhead.py [workload] [walkers]     -> one JSON line (also gpurun_out/step_overhead.json)"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import make_spec
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    workload = sys.argv[1] if len(sys.argv) > 1 else "canonical"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    spec, params = make_spec(workload, n, seed=1000)
    res = {"workload": workload, "walkers": n}
    T = 200
    for lanes in ("1", "2"):
        os.environ["WG_LANES"] = lanes
        os.environ["WG_STEP_LANES"] = lanes
        env = BatchedPhysicsEnv(spec, device="cuda:0", **params)
        A = max(1, env.batch.A)
        acts = (torch.rand((T, n, A), device="cuda:0") * 2 - 1).contiguous()
        env.run(acts, T, lanes=int(lanes))    # warm: the clocks up before anything is timed
        for s in range(10):
            env.step(acts[s])
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(st)
        for s in range(T):
            env.step(acts[s])
        e1.record(st)
        host = (time.perf_counter() - t0) / T
        torch.cuda.synchronize()
        closed = e0.elapsed_time(e1) / T
        env.run(acts, T, lanes=int(lanes))
        torch.cuda.synchronize()
        e0.record(st)
        env.run(acts, T, lanes=int(lanes))
        e1.record(st)
        torch.cuda.synchronize()
        res[f"lanes{lanes}"] = {"step_host_us": round(host * 1e6, 2), "step_closed_loop_us": round(closed * 1e3, 2),
                                "run_open_loop_us": round(e0.elapsed_time(e1) / T * 1e3, 2)}
        if lanes == "2":   # where the host time of step() goes
            pr = cProfile.Profile()
            pr.enable()
            for s in range(T):
                env.step(acts[s])
            pr.disable()
            torch.cuda.synchronize()
            buf = io.StringIO()
            pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(12)
            res["profile_lanes2"] = buf.getvalue().splitlines()[:40]
    del os.environ["WG_LANES"]
    del os.environ["WG_STEP_LANES"]
    line = json.dumps(res)
    print(line)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    open(os.path.join(ROOT, "gpurun_out", f"step_overhead_{workload}.json"), "w").write(line + "\n")


if __name__ == "__main__":
    main()
