"""Helper for test_gpu_parity.test_kernel_variants_agree (not a test module): runs a few uniform
batches through whichever step kernel the environment selects (WG_LEAN / WG_STREAM are read once per
process by libwalker_hip.so) and saves every output to an .npz."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cases():
    from walker_gym_amd.synthetic import canonical_walkers
    from walker_gym_amd.topologies import topology_spec
    from walker_gym_amd.walker import balance_spec
    import numpy as np
    pinned = canonical_walkers(700, seed=13)
    pinned["pinned"] = (np.random.default_rng(13).random(700 * 16) < 0.1).astype(np.uint8)
    pinned["vel"] = np.random.default_rng(14).normal(0, 1, (700 * 16, 3)).astype(np.float32)
    return [("canonical", canonical_walkers(1003, seed=11), dict(in3d=1), 8),   # 1003: a partial last wave
            ("balance", balance_spec(997), dict(in3d=0), 2),
            ("canonical2d", canonical_walkers(640, seed=12), dict(in3d=0, dampk=0.2, midform=0), 8),
            ("pinned_run2", pinned, dict(in3d=1, integrator=2), 8),
            ("g1_box2", topology_spec("box2", 997, 1), dict(in3d=0, midform=2, conmid=1), 4)]


def run(out_path):
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    res = {}
    for name, spec, params, A in cases():
        N = len(spec["mass_off"]) - 1
        acts = np.random.default_rng(len(name)).uniform(-1, 1, (25, N, A)).astype(np.float32)
        env = BatchedPhysicsEnv(spec, **params)
        o, r, d = env.rollout(acts)
        torch.cuda.synchronize()
        res[name + "_obs"] = o.cpu().numpy()
        res[name + "_rew"] = r.cpu().numpy()
        res[name + "_done"] = d.cpu().numpy()
        for f in ("pos", "vel", "acc", "muscle_x", "contact", "steps"):
            res[name + "_" + f] = (env.batch.steps if f == "steps" else getattr(env, f)).cpu().numpy()
    np.savez(out_path, **res)


if __name__ == "__main__":
    run(sys.argv[1])
