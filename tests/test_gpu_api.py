"""The drop-in API on the GPU against the reference's own env objects (tests/golden/api):

* walker_gym_amd.optimized_env.make_env / PhysicsEnv: np.random.seed -> construction (reset noise) -> seed(s) ->
  reset() -> step(a) x T returns the same observations (float64 arrays), float32 rewards, done flags (every done
  branch: max_steps, all-stopped after step 100, the 1,000-step rollout), info dicts and point states as
  gym/optimized_env.py's PhysicsEnv with the SURVEY §8(c) fixes;
* walker_gym_amd.env.Environment (G1): random.seed -> construction noise -> step(t) x 50 with varying t gives the
  states of gym/env.py's Environment, G1 friction included.
Tolerance: bit-exact everywhere (the energy's float32 ** 2 is libm powf, restated in walker_gym_amd/csrc/powf2.h).
"""
import glob
import os
import random

import numpy as np
import pytest

from api_replay import g1_creatures
from conftest import GOLDEN, gpu_available

pytestmark = pytest.mark.gpu
API = sorted(glob.glob(os.path.join(GOLDEN, "api", "api_*.npz")))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no ROCm GPU")


@pytest.mark.parametrize("path", API, ids=[os.path.basename(p) for p in API])
def test_physicsenv_facade_matches_reference(path):
    from walker_gym_amd.optimized_env import make_env
    z = np.load(path)
    np.random.seed(int(z["np_seed_init"]))
    env = make_env(str(z["env_id"]), in3d=bool(int(z["kwargs_in3d"])), dampk=float(z["kwargs_dampk"]),
                   rand_sigma=float(z["kwargs_rand_sigma"]), device="cuda:0")
    env.max_steps = int(z["max_steps"])
    assert env.seed(int(z["env_seed"])) == [int(z["env_seed"])]
    obs0 = env.reset()
    assert isinstance(obs0, np.ndarray) and obs0.dtype == np.float64
    np.testing.assert_array_equal(obs0, z["out_obs0"])
    T = z["actions"].shape[0]
    every = 10 if z["out_pos"].shape[0] != T else 1
    assert env.get_action_space()["shape"] == (z["actions"].shape[1],)
    assert env.get_observation_space()["shape"] == (z["out_obs0"].shape[0],)
    for t in range(T):
        obs, reward, done, info = env.step(z["actions"][t])
        assert isinstance(reward, np.float32) and reward == z["out_reward"][t], t
        assert isinstance(done, bool) and done == bool(z["out_done"][t]), t
        assert info["steps"] == z["out_steps"][t]
        assert isinstance(info["total_energy"], np.float32)
        assert info["total_energy"] == z["out_energy"][t], t
        if (t + 1) % every == 0:
            s = (t + 1) // every - 1
            np.testing.assert_array_equal(obs, z["out_obs"][s])
            assert info["centroid_position"] == list(z["out_centroid"][s])
            st = env._host_state()
            np.testing.assert_array_equal(st["pos"], z["out_pos"][s])
            np.testing.assert_array_equal(st["v"], z["out_vel"][s])
            np.testing.assert_array_equal(st["old_a"], z["out_acc"][s])


def test_g1_environment_facade_matches_reference():
    from walker_gym_amd.env import Environment
    z = np.load(os.path.join(GOLDEN, "api", "g1_env.npz"))
    random.seed(int(z["random_seed"]))
    env = Environment(g1_creatures(z["g1_names"]), in3d=bool(int(z["in3d"])), dampk=float(z["dampk"]),
                      randsigma=float(z["randsigma"]), device="cuda:0")
    np.testing.assert_array_equal(env._host_state()["v"], z["out_vel0"])
    for s, t in enumerate(z["ts"]):
        env.step(float(t))
        st = env._host_state()
        np.testing.assert_array_equal(st["pos"], z["out_pos"][s])
        np.testing.assert_array_equal(st["v"], z["out_vel"][s])
        np.testing.assert_array_equal(st["old_a"], z["out_acc"][s])
    # the point objects read the device state live (gym/engine.py Point attributes)
    p = env.creatures[0].phys[0]
    np.testing.assert_array_equal(p.pos, z["out_pos"][-1][0])


def test_make_env_unknown_id_raises():
    from walker_gym_amd.optimized_env import make_env
    with pytest.raises(ValueError, match="Unknown environment ID"):
        make_env("Walker-v9", device="cuda:0")


@pytest.mark.parametrize("args,head", [(["--steps", "60"], "Balance-v0: "), (["--env", "Box-v0", "--steps", "30"], "Box-v0: "),
                                       (["--g1", "leg2", "--steps", "20"], "leg2: 20 steps")])
def test_demo_runs(args, head):
    """BASELINE config 0 (one walker through the gym API, demo.py) runs end to end on the GPU stepper."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "demo.py")] + args, capture_output=True, text=True,
                       timeout=180, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    line = r.stdout.strip().splitlines()[-1]
    assert line.startswith(head), line
    assert "nan" not in line.lower(), line


def test_step_ranges_validates_every_range_before_launching():
    """wg_step_ranges checks every range's arguments before the first launch: a bad second range fails
    the call with no walker of the first range stepped."""
    import ctypes as C
    import numpy as np
    import torch
    from walker_gym_amd import _lib
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    env = BatchedPhysicsEnv(canonical_walkers(256, seed=3), device="cuda:0", in3d=1)
    before = env.pos.clone()
    steps0 = env.steps.clone()
    L = _lib.load()
    b = env.batch
    good, o = b.sub_struct(0, 128), env._outputs(env.obs[:128], env.reward[:128], env.done[:128])
    bad = b.sub_struct(128, 256)
    bad.M = 0                                   # invalid: the second range's own checks fail
    rng = (_lib.WgRange * 2)()
    rng[0].batch, rng[0].outputs, rng[0].stream = C.pointer(good), C.pointer(o), torch.cuda.current_stream().cuda_stream
    rng[1].batch, rng[1].outputs, rng[1].stream = C.pointer(bad), C.pointer(o), torch.cuda.current_stream().cuda_stream
    evs = [torch.cuda.Event() for _ in range(2)]
    for e in evs:
        e.record()
    events = (C.c_void_p * 2)(*[e.cuda_event for e in evs])
    rc = L.wg_step_ranges(rng, 2, C.byref(env._pstruct), None, 0, 0, events)
    torch.cuda.synchronize()
    assert rc == _lib.WG_EINVAL
    assert torch.equal(env.pos, before) and torch.equal(env.steps, steps0)


@pytest.mark.parametrize("workload", ["canonical", "balance2d"])
def test_survey_signature_entry_points_bit_exact(workload):
    """SURVEY §8(b)'s declared signatures (ABI 13): wg_step_simple(batch, action, params, n_steps, stream) for T steps
    with [T, N, A] actions in one call, then wg_observe_simple(batch, cfg, obs, reward, done, centroid, energy, stream),
    bit-identical to the same walkers stepped by BatchedPhysicsEnv.run (wg_run_ranges) — state, step counters and
    every output; a ragged batch is refused."""
    import ctypes as C
    import torch
    from walker_gym_amd import _lib
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers, ragged_walkers
    from walker_gym_amd.walker import balance_spec
    spec, kw = (canonical_walkers(640, seed=11), dict(in3d=1)) if workload == "canonical" else (balance_spec(640), dict(in3d=0))
    a_env = BatchedPhysicsEnv(spec, device="cuda:0", **kw)
    b_env = BatchedPhysicsEnv(spec, device="cuda:0", **kw)
    T, N, A = 25, a_env.N, a_env.batch.A
    g = torch.Generator(device="cuda:0").manual_seed(5)
    acts = (torch.rand((T, N, A), generator=g, device="cuda:0") * 2 - 1).contiguous()
    a_env.run(acts, T)
    L = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    assert L.wg_step_simple(C.byref(b_env.batch.struct), acts.data_ptr(), C.byref(b_env._pstruct), T, st) == 0
    obs = torch.full((N, a_env.obs_dim), -7.0, device="cuda:0")
    rew = torch.empty(N, device="cuda:0")
    done = torch.empty(N, dtype=torch.uint8, device="cuda:0")
    cen = torch.empty((N, 3), device="cuda:0")
    en = torch.empty(N, device="cuda:0")
    assert L.wg_observe_simple(C.byref(b_env.batch.struct), C.byref(b_env._pstruct), obs.data_ptr(), rew.data_ptr(),
                               done.data_ptr(), cen.data_ptr(), en.data_ptr(), st) == 0
    torch.cuda.synchronize()
    for name in ("pos", "vel", "acc", "muscle_x", "steps"):
        assert torch.equal(getattr(a_env, name), getattr(b_env, name)), name
    bits = lambda t: t.contiguous().view(torch.int32)
    assert torch.equal(bits(obs), bits(a_env.obs))
    assert torch.equal(bits(rew), bits(a_env.reward)) and torch.equal(done.bool(), a_env.done)
    assert torch.equal(bits(cen), bits(a_env.centroid)) and torch.equal(bits(en), bits(a_env.energy))
    r_env = BatchedPhysicsEnv(ragged_walkers(64, seed=2, mmin=4, mmax=12), device="cuda:0", in3d=1)
    assert L.wg_step_simple(C.byref(r_env.batch.struct), None, C.byref(r_env._pstruct), 1, st) == _lib.WG_EINVAL
    assert b"uniform batches only" in L.wg_last_error()


@pytest.mark.parametrize("workload", ["canonical", "ragged", "balance2d", "chain"])
def test_time_launches_steps_as_run(workload):
    """wg_time_step (ABI 14, bench.py's roofline): the same steps as run(lanes=1) — every step kernel (lean, wave, NE = 1
    and workgroup kernels) launched through hipExtLaunchKernel with its own start / end events — bit-identical state
    and outputs, and a positive mean kernel duration."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers, chain_walkers, ragged_walkers
    from walker_gym_amd.walker import balance_spec
    spec, kw = {"canonical": (canonical_walkers(640, seed=4), dict(in3d=1)),
                "ragged": (ragged_walkers(300, seed=4, mmin=4, mmax=32), dict(in3d=1)),
                "balance2d": (balance_spec(640), dict(in3d=0)),
                "chain": (chain_walkers(40, 20, seed=4), dict(in3d=1, g=0.0, ground=-1.0e6, pair_mode=1))}[workload]
    a_env = BatchedPhysicsEnv(spec, device="cuda:0", **kw)
    b_env = BatchedPhysicsEnv(spec, device="cuda:0", **kw)
    T, N, A = 6, a_env.N, max(1, a_env.batch.A)
    g = torch.Generator(device="cuda:0").manual_seed(9)
    acts = (torch.rand((T, N, A), generator=g, device="cuda:0") * 2 - 1).contiguous()
    a_env.run(acts, T, lanes=1)
    ms = b_env.time_launches(acts, T)
    torch.cuda.synchronize()
    assert 0.0 < ms < 1000.0
    bits = lambda t: t.contiguous().view(torch.int32) if t.dtype == torch.float32 else t
    for name in ("pos", "vel", "acc", "muscle_x", "steps", "obs", "reward", "done", "centroid", "energy"):
        assert torch.equal(bits(getattr(a_env, name)), bits(getattr(b_env, name))), name
