"""BASELINE config 4 at its full size on the one GPU a box has: 524,288 canonical walkers
sharded over 8 ranks — the shard sizes, per-rank batches and rollout-end gather of the 8 x MI355X run — launched by
torch.distributed.run as 8 processes on cuda:0 over gloo (tests/config4_rank.py), plus an uneven variant with
524,287 walkers (shards of 65,536 and 65,535).  Each rank steps its shard T times through the HIP kernel exactly as
bench.py's timed rollout does (two walker ranges, per-step records); the gathered final observations, per-step
rewards / done flags / energies and final positions must be bitwise equal to the whole batch stepped by one
process, and the walkers on either side of every shard boundary (plus the first and last) bitwise equal to the CPU
oracle.  Only RCCL across GPUs is left to the driver's 8-GPU run."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
WORLD = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


@pytest.mark.parametrize("n_total", [8 * 65536, 8 * 65536 - 1])
def test_config4_eight_ranks_on_one_gpu(tmp_path, n_total):
    if not gpu_available():
        pytest.skip("no ROCm GPU")
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.distributed import shard_bounds, shard_spec
    from walker_gym_amd.synthetic import canonical_walkers
    T = 3
    spec = canonical_walkers(n_total, seed=44)
    acts = np.random.default_rng(44).uniform(-1, 1, (T, n_total, 8)).astype(np.float32)
    spec_path, out = str(tmp_path / "spec.npz"), str(tmp_path / "gathered.npz")
    np.savez(spec_path, n_total=n_total, T=T, acts=acts, **spec)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={WORLD}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "config4_rank.py"),
           spec_path, out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    g = np.load(out)
    assert int(g["world"]) == WORLD
    sizes = [b - a for a, b in (shard_bounds(n_total, WORLD, k) for k in range(WORLD))]
    assert sum(sizes) == n_total and max(sizes) - min(sizes) == (0 if n_total % WORLD == 0 else 1)

    # the whole batch in one process, the same path (two walker ranges, per-step records)
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    dv = "cuda:0"
    rec = {"reward": torch.empty((T, n_total), dtype=torch.float32, device=dv),
           "done": torch.empty((T, n_total), dtype=torch.uint8, device=dv),
           "energy": torch.empty((T, n_total), dtype=torch.float32, device=dv),
           "centroid": torch.empty((T, n_total, 3), dtype=torch.float32, device=dv)}
    env.run(torch.from_numpy(acts).to(dv), T, lanes=2, record=rec)
    torch.cuda.synchronize()
    one = {"obs": env.obs.cpu().numpy(), "reward": rec["reward"].cpu().numpy(), "done": rec["done"].cpu().numpy(),
           "energy": rec["energy"].cpu().numpy(), "pos": env.pos.reshape(n_total, -1).cpu().numpy()}
    for k, v in one.items():
        assert g[k].shape == v.shape, (k, g[k].shape, v.shape)
        assert np.array_equal(_bits(g[k]), _bits(v)), k
    del env

    # the oracle on the walkers either side of every shard boundary, the first and the last ones
    bounds = [shard_bounds(n_total, WORLD, k)[0] for k in range(1, WORLD)]
    chunks = [(0, 3)] + [(b - 2, b + 2) for b in bounds] + [(n_total - 3, n_total)]
    for a, b in chunks:
        orc = Oracle(shard_spec(spec, a, b), dict(in3d=1))
        for t in range(T):
            ref = orc.step(acts[t, a:b])
            assert np.array_equal(_bits(one["reward"][t, a:b]), _bits(ref["reward"])), (a, t)
            assert np.array_equal(one["done"][t, a:b], ref["done"]), (a, t)
            assert np.array_equal(_bits(one["energy"][t, a:b]), _bits(ref["energy"])), (a, t)
        assert np.array_equal(_bits(one["obs"][a:b]), _bits(ref["obs"])), a
        assert np.array_equal(_bits(one["pos"][a:b].reshape(-1, 3)), _bits(orc.pos)), a
