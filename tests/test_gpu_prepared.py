"""BatchedPhysicsEnv.prepare_run (run()'s C arguments built once; bench.py times the K steps as one C call) and the
round-4 ADVICE items on the env's output bookkeeping: a prepared run equals run() bit for bit, refuses to run after
the env's buffers change, and info() leaves out what a record / info=False run did not write."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no ROCm GPU")


def _bits(t):
    return t.detach().cpu().contiguous().numpy().view(np.uint8)


@pytest.mark.parametrize("kind,lanes", [("canonical", 1), ("canonical", 2), ("ragged", 2)])
def test_prepared_run_equals_run(kind, lanes):
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers, ragged_walkers
    N, T = 9000, 6
    spec = canonical_walkers(N, seed=12) if kind == "canonical" else ragged_walkers(N, seed=13, mmin=4, mmax=32)
    a = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    b = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    acts = (torch.rand((T, N, a.batch.A), generator=torch.Generator(device="cuda:0").manual_seed(5), device="cuda:0")
            * 2 - 1).contiguous()
    a.run(acts, T, lanes=lanes)
    a.run(acts, T, lanes=lanes)
    prep = b.prepare_run(acts, T, lanes=lanes)
    prep()
    prep()                                   # the same steps again, from the advanced state
    torch.cuda.synchronize()
    for name in ("pos", "vel", "acc", "obs", "reward", "done", "centroid", "energy", "muscle_x", "steps"):
        assert np.array_equal(_bits(getattr(a, name)), _bits(getattr(b, name))), name
    assert torch.equal(a.info()["steps"], b.info()["steps"])
    b.set_params(dampk=0.5)
    with pytest.raises(RuntimeError):
        prep()


def test_record_run_marks_info_stale_and_needs_steps():
    """after run(record=...) the env's centroid / energy / extras are not this run's: info() leaves them out
    until the next step(); record with n_steps = 0 is refused up front."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    N, T = 512, 3
    env = BatchedPhysicsEnv(canonical_walkers(N, seed=3), device="cuda:0", in3d=1, info_extras=True)
    acts = torch.zeros((T, N, env.batch.A), device="cuda:0")
    rec = {"reward": torch.empty((T, N), device="cuda:0"), "done": torch.empty((T, N), dtype=torch.uint8,
                                                                                device="cuda:0")}
    env.run(acts, T, record=rec)
    info = env.info()
    assert set(info) == {"steps"}
    assert torch.equal(info["steps"], torch.full((N,), T, dtype=torch.int32, device="cuda:0"))
    env.step(acts[0])
    assert {"steps", "centroid_position", "total_energy", "momentum", "nonfinite"} <= set(env.info())
    with pytest.raises(ValueError):
        env.run(acts[:1], 0, record={"reward": rec["reward"][:0], "done": rec["done"][:0]})


def test_enable_info_extras_keeps_the_other_outputs():
    """enabling the extras allocates only momentum and nonfinite; the obs / reward tensors a caller holds
    stay the env's live outputs."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    env = BatchedPhysicsEnv(canonical_walkers(256, seed=4), device="cuda:0", in3d=1)
    obs, rew, done, _ = env.step(torch.zeros((256, env.batch.A), device="cuda:0"))
    before = obs.clone()
    env.enable_info_extras()
    obs2, rew2, _, info = env.step(torch.ones((256, env.batch.A), device="cuda:0") * 0.5)
    assert obs2 is obs and rew2 is rew
    assert not torch.equal(obs, before)       # the held tensor saw the second step
    assert info["momentum"].shape == (256, 3) and info["nonfinite"].dtype == torch.bool
