"""Rank program of test_gpu_distributed.py's RCCL test (not a test module): launched by torch.distributed.run with
ONE rank on cuda:0 over the nccl backend (= RCCL on ROCm), the transport the 8-GPU run (BASELINE config 4) uses.
It steps a canonical shard through the HIP kernel, then drives walker_gym_amd.distributed.gather_rollout on DEVICE
tensors exactly as bench.py does at rollout end, with n_total given and omitted, on an odd row count and on each
output dtype of a rollout (f32 obs / reward, u8 done).  Every gathered tensor must be bitwise equal to its input
(one rank: the gather is the identity).  Results go to the JSON file named on the command line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(out_path: str) -> None:
    import torch
    import torch.distributed as dist
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.distributed import gather_rollout
    from walker_gym_amd.synthetic import canonical_walkers
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    res = {"backend": dist.get_backend(), "world": dist.get_world_size(), "checks": {}}
    n, T = 1001, 4
    env = BatchedPhysicsEnv(canonical_walkers(n, seed=5), device=dev, in3d=1)
    acts = torch.rand((T, n, 8), generator=torch.Generator(device=dev).manual_seed(3), device=dev) * 2 - 1
    obs, rew, done = env.rollout(acts)
    cases = {
        "obs_rows_n_total": (obs.transpose(0, 1).contiguous(), n),
        "obs_rows_sizes_gathered": (obs.transpose(0, 1).contiguous(), None),
        "reward_rows": (rew.transpose(0, 1).contiguous(), n),
        "done_rows_u8": (done.transpose(0, 1).contiguous(), n),
        "final_obs": (env.obs, None),
        "odd_rows_3": (env.obs[:3].contiguous(), 3),
    }
    for name, (t, nt) in cases.items():
        g = gather_rollout(t, n_total=nt)
        torch.cuda.synchronize()
        res["checks"][name] = {
            "device": str(g.device), "shape_ok": tuple(g.shape) == tuple(t.shape), "dtype_ok": g.dtype == t.dtype,
            "bitwise": bool(torch.equal(g.view(torch.uint8) if g.dtype != torch.uint8 else g,
                                        t.view(torch.uint8) if t.dtype != torch.uint8 else t))}
    # the learner-only gather (dist.gather to rank 0, bench.py's default rollout-end collective)
    for name, (t, nt) in {"root_final_obs": (env.obs, n), "root_reward_steps": (rew, n)}.items():
        g = gather_rollout(t, n_total=nt, dim=1 if name == "root_reward_steps" else 0, dst=0)
        torch.cuda.synchronize()
        res["checks"][name] = {
            "device": str(g.device), "shape_ok": tuple(g.shape) == tuple(t.shape), "dtype_ok": g.dtype == t.dtype,
            "bitwise": bool(torch.equal(g.view(torch.uint8), t.contiguous().view(torch.uint8)))}
    # a wrong n_total is refused before any collective (shard_bounds disagrees with the local row count)
    try:
        gather_rollout(env.obs, n_total=n + 1)
        res["wrong_n_total_refused"] = False
    except ValueError:
        res["wrong_n_total_refused"] = True
    dist.barrier()
    with open(out_path, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
