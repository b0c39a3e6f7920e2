"""World-size-2/3 gloo tests of the sharded path on the CPU: each rank steps its contiguous
walker shard (here with the CPU oracle standing in for the GPU kernel — the plumbing under test is the shard
split and the rollout-end gather, including uneven shards), gathers observations, and the result equals the
unsharded batch.  The same path through the HIP kernel is test_gpu_distributed.py; bench.py's own rank
launcher is test_bench_launcher.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from walker_gym_amd.distributed import shard_bounds, shard_spec


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, T, out_q, by_size, pipelined=False):
    import torch
    import torch.distributed as dist
    from oracle.oracle import Oracle
    from walker_gym_amd.distributed import gather_rollout, gather_rollout_async
    from walker_gym_amd.synthetic import canonical_walkers
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = canonical_walkers(n_total, seed=4)
    acts = np.random.default_rng(4).uniform(-1, 1, (T, n_total, 8)).astype(np.float32)
    a, b = shard_bounds(n_total, world, rank)
    orc = Oracle(shard_spec(spec, a, b), dict(in3d=1))
    obs, rew, done = None, [], []
    for t in range(T):
        o = orc.step(acts[t, a:b])
        obs = o["obs"]
        rew.append(o["reward"]); done.append(o["done"])
    if pipelined:
        # bench.py's pipelined gather: issue the gather of this rollout's final observations, keep stepping (the next
        # rollout; the oracle writes fresh arrays, so the gathered buffer is not touched), then wait
        h = gather_rollout_async(torch.from_numpy(obs.copy()), n_total=None if by_size else n_total)
        for t in range(2):
            orc.step(acts[t, a:b])
        full = h.wait()
    else:
        full = gather_rollout(torch.from_numpy(obs), n_total=None if by_size else n_total)
    # the per-step records of SURVEY §8(e) ([T, n_r] -> [T, N], dim 1), as bench.py's rollout gather sends them
    rew_full = gather_rollout(torch.from_numpy(np.stack(rew)), n_total=None if by_size else n_total, dim=1)
    done_full = gather_rollout(torch.from_numpy(np.stack(done)), n_total=None if by_size else n_total, dim=1)
    # the learner-only form (dist.gather to one rank; bench.py's default): the last rank receives, the others get None
    root = world - 1
    obs_root = gather_rollout(torch.from_numpy(obs), n_total=None if by_size else n_total, dst=root)
    rew_root = gather_rollout(torch.from_numpy(np.stack(rew)), n_total=None if by_size else n_total, dim=1, dst=root)
    if rank != root:
        assert obs_root is None and rew_root is None
    else:
        assert np.array_equal(obs_root.numpy(), full.numpy()) and np.array_equal(rew_root.numpy(), rew_full.numpy())
    if rank == 0:
        out_q.put((full.numpy(), rew_full.numpy(), done_full.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds_cover():
    for n in (0, 1, 7, 65536, 524288):
        for w in (1, 2, 3, 8):
            rs = [shard_bounds(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


@pytest.mark.parametrize("world,n_total,by_size,pipelined", [(2, 64, False, False), (2, 65, False, False),
                                                             (3, 65, True, False), (2, 65, False, True),
                                                             (8, 1003, False, False), (8, 1003, True, False)])
def test_gloo_matches_single_process(world, n_total, by_size, pipelined):
    """Even and uneven shards (65 walkers: ranks of 33/32 or 22/22/21; config 4's world of 8 with 1,003 walkers:
    ranks of 126 / 125), lengths from shard_bounds or gathered; the pipelined form (gather issued, more steps, then
    waited) gathers the same rows; the per-step rewards and done flags gather along their walker axis."""
    from oracle.oracle import Oracle
    from walker_gym_amd.synthetic import canonical_walkers
    T = 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, T, q, by_size, pipelined))
             for r in range(world)]
    for p in procs:
        p.start()
    got, got_rew, got_done = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spec = canonical_walkers(n_total, seed=4)
    acts = np.random.default_rng(4).uniform(-1, 1, (T, n_total, 8)).astype(np.float32)
    orc = Oracle(spec, dict(in3d=1))
    rew, done = [], []
    for t in range(T):
        o = orc.step(acts[t])
        ref = o["obs"]
        rew.append(o["reward"]); done.append(o["done"])
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)
    assert np.array_equal(got_rew.view(np.uint32), np.stack(rew).view(np.uint32))
    assert np.array_equal(got_done, np.stack(done))
