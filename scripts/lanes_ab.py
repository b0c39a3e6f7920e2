"""A/B of BatchedPhysicsEnv.run lanes (walker ranges on separate streams) on the bench workload, one process:
per lanes value, wall time per step over the same timed region bench.py uses; then bit-equality of the
state after lanes=L vs lanes=1 from the same start."""
import sys
import time

import torch

sys.path.insert(0, ".")
from bench import make_spec  # noqa: E402
from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
WORKLOAD = sys.argv[2] if len(sys.argv) > 2 else "canonical"
STEPS = 500
spec, params = make_spec(WORKLOAD, N, seed=1000)
env = BatchedPhysicsEnv(spec, device="cuda:0", **params)
gen = torch.Generator(device="cuda:0")
gen.manual_seed(7)
acts = (torch.rand((STEPS, N, env.batch.A), generator=gen, device="cuda:0") * 2 - 1).contiguous()
sd0 = env.batch.state_dict()
res = {}
for rep in range(5):
    for lanes in (1, 2, 4):
        env.run(acts[:30], 30, lanes=lanes)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        env.run(acts, STEPS, lanes=lanes)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / STEPS * 1e6
        res.setdefault(lanes, []).append(us)
        print(f"rep {rep} lanes {lanes}: {us:.2f} us/step  {N / us * 1e6:.3e} env-steps/s", flush=True)
for lanes in (2, 4):
    env.batch.load_state_dict(sd0)
    env.run(acts[:50], 50, lanes=1)
    a = {k: v.clone() for k, v in env.batch.state_dict().items()}
    o1 = env.obs.clone()
    env.batch.load_state_dict(sd0)
    env.run(acts[:50], 50, lanes=lanes)
    torch.cuda.synchronize()
    b = env.batch.state_dict()
    same = all(torch.equal(a[k], b[k]) for k in a) and torch.equal(o1, env.obs)
    print(f"lanes {lanes} bit-identical to lanes 1: {same}")
import statistics
print('min', {k: round(min(v), 2) for k, v in res.items()}, 'median', {k: round(statistics.median(v), 2) for k, v in res.items()})
