"""Rank program of test_distributed_gpu (not a test module): launched by torch.distributed.run with 2+ ranks
that share cuda:0 over gloo.  Every rank steps its contiguous shard of one seeded canonical batch through the
HIP kernel (BatchedPhysicsEnv.rollout), then the per-step observations / rewards / done flags are gathered
with gather_rollout; rank 0 saves the gathered arrays to the .npz named on the command line."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(out_path: str, n_total: int, T: int) -> None:
    import torch
    import torch.distributed as dist
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.distributed import gather_rollout, shard_bounds, shard_spec
    from walker_gym_amd.synthetic import canonical_walkers
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    spec = canonical_walkers(n_total, seed=21)
    acts = np.random.default_rng(21).uniform(-1, 1, (T, n_total, 8)).astype(np.float32)
    a, b = shard_bounds(n_total, world, rank)
    env = BatchedPhysicsEnv(shard_spec(spec, a, b), device="cuda:0", in3d=1)
    obs, rew, done = env.rollout(acts[:, a:b])
    torch.cuda.synchronize()
    # gloo gathers host tensors: [T, n, ...] -> walker-major rows, gathered, back to [T, N, ...]
    g = {}
    for name, t in (("obs", obs), ("reward", rew), ("done", done), ("pos", env.pos.reshape(b - a, -1))):
        loc = t.transpose(0, 1).contiguous().cpu() if name != "pos" else t.cpu()
        full = gather_rollout(loc, n_total=n_total)
        g[name] = np.ascontiguousarray((full.transpose(0, 1) if name != "pos" else full).numpy())
    if rank == 0:
        np.savez(out_path, world=world, **g)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))
