#!/usr/bin/env python3
"""Host time of one BatchedPhysicsEnv.run() call (profiling aid): the Python + C work before and while a run's launches
are issued, which the GPU waits through at the start of a timed region.  Canonical 65,536 walkers, two walker ranges,
bench.py's record buffers; each call is timed on the host after a full sync (so the launch queue is empty), with
n_steps 1 and 20.  Writes gpurun_out/run_overhead.json."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import make_spec
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    n, dev = 65536, "cuda:0"
    spec, params = make_spec("canonical", n, seed=1000)
    env = BatchedPhysicsEnv(spec, device=dev, **params)
    res = {}
    for K in (1, 20):
        acts = (torch.rand((K, n, env.batch.A), device=dev) * 2 - 1).contiguous()
        rec = {"reward": torch.empty((K, n), device=dev), "done": torch.empty((K, n), dtype=torch.bool, device=dev),
               "energy": torch.empty((K, n), device=dev), "centroid": torch.empty((K, n, 3), device=dev)}
        for issue in ("inter", "seq"):
            os.environ["WG_RANGE_ISSUE"] = issue
            ts = []
            for i in range(60):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                env.run(acts, K, lanes=2, record=rec)
                ts.append((time.perf_counter() - t0) * 1e6)
            torch.cuda.synchronize()
            res[f"{issue}_K{K}_us"] = round(statistics.median(ts[10:]), 1)
    print(json.dumps(res))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "run_overhead.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
