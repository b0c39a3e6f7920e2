"""Rank program of test_gpu_config4 (not a test module): BASELINE config 4's workload — 524,288 canonical walkers
sharded over 8 ranks — rehearsed on the one GPU of the box.  Launched by torch.distributed.run with 8 ranks that
share cuda:0 over gloo (RCCL cannot put two ranks on one GPU).  Each rank loads its contiguous shard
(shard_bounds) of the seeded batch the parent wrote, steps it T times through the HIP kernel exactly as bench.py's
timed rollout does (BatchedPhysicsEnv.run with two walker ranges, per-step reward / done / energy / centroid
recorded), then the rollout-end gather of SURVEY §8(e) runs: the final observations [N, D] and the per-step
rewards and done flags [T, N] (distributed.gather_rollout, dim 1 for the per-step records).  Rank 0 saves the
gathered arrays to the .npz named on the command line."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(spec_path: str, out_path: str) -> None:
    import torch
    import torch.distributed as dist
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.distributed import gather_rollout, shard_bounds, shard_spec
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    z = np.load(spec_path, mmap_mode="r")
    n_total, T = int(z["n_total"]), int(z["T"])
    spec = {k: z[k] for k in z.files if k not in ("n_total", "T", "acts")}
    a, b = shard_bounds(n_total, world, rank)
    env = BatchedPhysicsEnv(shard_spec(spec, a, b), device="cuda:0", in3d=1)
    n = b - a
    acts = torch.from_numpy(np.ascontiguousarray(z["acts"][:, a:b])).to("cuda:0")
    rec = {"reward": torch.empty((T, n), dtype=torch.float32, device="cuda:0"),
           "done": torch.empty((T, n), dtype=torch.uint8, device="cuda:0"),
           "energy": torch.empty((T, n), dtype=torch.float32, device="cuda:0"),
           "centroid": torch.empty((T, n, 3), dtype=torch.float32, device="cuda:0")}
    env.run(acts, T, lanes=2, record=rec)
    torch.cuda.synchronize()
    # gloo gathers host tensors
    g = {"obs": gather_rollout(env.obs.cpu(), n_total=n_total),
         "reward": gather_rollout(rec["reward"].cpu(), n_total=n_total, dim=1),
         "done": gather_rollout(rec["done"].cpu(), n_total=n_total, dim=1),
         "energy": gather_rollout(rec["energy"].cpu(), n_total=n_total, dim=1),
         "pos": gather_rollout(env.pos.reshape(n, -1).cpu(), n_total=n_total)}
    if rank == 0:
        np.savez(out_path, world=world, **{k: v.numpy() for k, v in g.items()})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
