"""Ragged batches on the GPU, through the C ABI:

* the wave kernel (wg_batch.ragged = 2: walkers stored in best-fit wave-tile order, tiles planned by wg_plan_waves) is
  bitwise equal to the workgroup kernel running the same plan (WG_LEAN=0), and both to the oracle with the
  outputs back in the caller's walker order;
* pair forces (gym/engine.py:114-147 per walker) on the workgroup kernel: ragged batches and uniform walkers
  whose M does not divide 64 match the oracle bit for bit;
* reset noise and masks given in the caller's order land on the right (sorted) walkers; wg_reset_noise keeps a
  2D walker's v.z = -0.0.
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no ROCm GPU")


def _rollout(spec, params, acts, lean=True):
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    if not lean:
        os.environ["WG_LEAN"] = "0"
    try:
        env = BatchedPhysicsEnv(spec, device="cuda:0", **params)
        o, r, d = env.rollout(acts)
        torch.cuda.synchronize()
        out = [o, r, d, env.pos, env.vel, env.acc, env.muscle_x, env.contact, env.steps, env.centroid, env.energy]
        return env, [t.cpu().numpy() for t in out]
    finally:
        os.environ.pop("WG_LEAN", None)


@pytest.mark.parametrize("params", [dict(in3d=1, dampk=0.3), dict(in3d=0, midform=2, conmid=1),
                                    dict(in3d=1, integrator=2, midform=0)])
def test_wave_kernel_equals_workgroup_kernel(params):
    from walker_gym_amd.synthetic import ragged_walkers
    N = 3001
    spec = ragged_walkers(N, seed=41, mmin=2, mmax=48, string_frac=0.1)
    A = int(np.max(spec["n_muscles"]))
    acts = np.random.default_rng(41).uniform(-1, 1, (12, N, A)).astype(np.float32)
    env, wave = _rollout(spec, params, acts, lean=True)
    assert env.batch.ragged_kind == 2 and env.batch.row is not None
    _, wg = _rollout(spec, params, acts, lean=False)
    for x, y in zip(wave, wg):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8))


def test_wave_kernel_vs_oracle_caller_order():
    """63 walkers of descending size (the sort reverses them); one walker of M = 64 fills a wave alone."""
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import ragged_walkers
    parts = [ragged_walkers(1, seed=100 + i, mmin=m, mmax=m) for i, m in enumerate(range(64, 1, -1))]
    from walker_gym_amd.walker import concat_specs
    spec = concat_specs(parts)
    N = len(spec["mass_off"]) - 1
    A = int(np.max(spec["n_muscles"]))
    acts = np.random.default_rng(5).uniform(-1, 1, (15, N, A)).astype(np.float32)
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    assert env.batch.ragged_kind == 2
    orc = Oracle(spec, dict(in3d=1))
    for t in range(15):
        obs, rew, done, info = env.step(acts[t])
        ref = orc.step(acts[t])
    torch.cuda.synchronize()
    assert np.array_equal(env.pos.cpu().numpy(), orc.pos)
    assert np.array_equal(obs.cpu().numpy(), ref["obs"])
    assert np.array_equal(rew.cpu().numpy(), ref["reward"])
    assert np.array_equal(info["centroid_position"].cpu().numpy(), ref["centroid"])
    assert np.array_equal(env.muscle_x.cpu().numpy(), orc.mx)


def test_wave_kernel_dense_walkers_vs_oracle():
    """Walkers of more than 128 springs (M = 64, K = 200: the wave kernel's incidence entries no longer fit one byte,
    so the tile keeps two-byte entries) mixed with small ones, against the oracle in the caller's order."""
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers, ragged_walkers
    from walker_gym_amd.walker import concat_specs
    spec = concat_specs([canonical_walkers(3, seed=61, M=64, K=200, A=12), ragged_walkers(40, seed=62, mmin=3, mmax=20),
                         canonical_walkers(2, seed=63, M=49, K=150, A=9)])
    N = len(spec["mass_off"]) - 1
    A = int(np.max(spec["n_muscles"]))
    acts = np.random.default_rng(64).uniform(-1, 1, (12, N, A)).astype(np.float32)
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    assert env.batch.ragged_kind == 2 and env.launch_geometry()["threads"] > 0
    orc = Oracle(spec, dict(in3d=1))
    for t in range(12):
        obs, rew, done, info = env.step(acts[t])
        ref = orc.step(acts[t])
    torch.cuda.synchronize()
    assert np.array_equal(env.pos.cpu().numpy().view(np.uint32), orc.pos.view(np.uint32))
    assert np.array_equal(env.vel.cpu().numpy().view(np.uint32), orc.vel.view(np.uint32))
    assert np.array_equal(obs.cpu().numpy().view(np.uint32), ref["obs"].view(np.uint32))
    assert np.array_equal(rew.cpu().numpy().view(np.uint32), ref["reward"].view(np.uint32))
    assert np.array_equal(env.muscle_x.cpu().numpy(), orc.mx)


@pytest.mark.parametrize("pair_mode", [7, 31, "4_subset"])
@pytest.mark.parametrize("case", ["ragged", "uniform_M13", "uniform_M100", "uniform_M100_wide"])
def test_pair_forces_workgroup_kernel_vs_oracle(case, pair_mode):
    """4_subset: Point.bounce(k, other=<list>) with random caller / list bits per point (wg_batch.bounce_set)."""
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers, ragged_walkers
    from walker_gym_amd.topologies import topology_spec
    rng = np.random.default_rng(7)
    if case == "ragged":
        spec = ragged_walkers(600, seed=7, mmin=3, mmax=40)
    elif case == "uniform_M13":
        spec = topology_spec("insect", 500, 1)
    elif case == "uniform_M100":
        spec = canonical_walkers(40, seed=7, M=100, K=180, A=10)
    else:   # enough walkers for 512-thread workgroups of 5 walkers (wg_launch_geometry checked below)
        spec = canonical_walkers(2600, seed=8, M=100, K=180, A=10)
    P = int(spec["mass_off"][-1])
    spec["charge"] = rng.uniform(-3, 3, P)
    spec["radius"] = rng.uniform(0.5, 2.0, P)
    if pair_mode == "4_subset":
        pair_mode = 4
        spec["bounce_set"] = rng.integers(0, 4, P).astype(np.uint8)
    N = len(spec["mass_off"]) - 1
    A = max(1, int(np.max(spec["n_muscles"])))
    params = dict(in3d=1, pair_mode=pair_mode, pair_g=500.0, pair_k=2.0e3, bounce_k=400.0)
    env = BatchedPhysicsEnv(spec, device="cuda:0", **params)
    # pair forces run on the workgroup kernel, on a plan of its own (not the wave tiles)
    assert env.batch.ragged_kind == (1 if case == "ragged" else 0), env.batch.ragged_kind
    if case == "uniform_M100_wide":
        info = env.launch_geometry()
        assert info["threads"] == 512 and info["walkers_per_block"] == 5, info
    orc = Oracle(spec, params)
    T = 4 if case == "uniform_M100_wide" else 10
    acts = rng.uniform(-1, 1, (T, N, A)).astype(np.float32)
    for t in range(T):
        obs, rew, done, info = env.step(acts[t])
        ref = orc.step(acts[t])
    torch.cuda.synchronize()
    assert np.array_equal(env.pos.cpu().numpy(), orc.pos, equal_nan=True)
    assert np.array_equal(env.vel.cpu().numpy(), orc.vel, equal_nan=True)
    assert np.array_equal(obs.cpu().numpy(), ref["obs"], equal_nan=True)
    assert np.array_equal(env.batch.caller("radius").cpu().numpy(), orc.radius)


def test_ragged_reset_noise_and_mask_in_caller_order():
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import ragged_walkers
    N = 500
    spec = ragged_walkers(N, seed=9, mmin=2, mmax=30)
    P = int(spec["mass_off"][-1])
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    assert env.batch.row is not None
    noise = np.random.default_rng(9).normal(0, 0.5, (P, 3)).astype(np.float32)
    orc = Oracle(spec, dict(in3d=1))
    env.reset(noise)
    orc.reset(noise)
    torch.cuda.synchronize()
    assert np.array_equal(env.vel.cpu().numpy(), orc.vel)
    # masked reset: only odd caller walkers
    A = int(np.max(spec["n_muscles"]))
    acts = np.random.default_rng(10).uniform(-1, 1, (3, N, A)).astype(np.float32)
    for t in range(3):
        env.step(acts[t])
    mask = (np.arange(N) % 2).astype(np.uint8)
    v_before = env.vel.cpu().numpy()
    env.reset(noise, mask=mask)
    torch.cuda.synchronize()
    v_after = env.vel.cpu().numpy()
    steps = env.steps.cpu().numpy()
    wid = np.repeat(np.arange(N), np.diff(spec["mass_off"]))
    sel = mask[wid] == 1
    assert np.array_equal(v_after[~sel], v_before[~sel])
    assert np.array_equal(v_after[sel], (v_before + noise)[sel])
    assert np.array_equal(steps, np.where(mask == 1, 0, 3))


def test_reset_noise_2d_keeps_negative_zero():
    """wg_reset_noise skips noise components that are exactly +0.0: a 2D caller's z = +0.0 leaves v.z = -0.0 as it
    is, bit for bit the same as wg_reset with in3d = 0 (PhysicsEnv.reset adds x and y only in 2D)."""
    import torch
    from walker_gym_amd import _lib
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.walker import balance_spec
    spec = balance_spec(256)
    spec["vel"] = np.zeros_like(spec["vel"])
    spec["vel"][:, 2] = -0.0
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=0)
    noise = torch.randn((256 * 4, 3), generator=torch.Generator(device="cuda:0").manual_seed(3), device="cuda:0")
    noise[:, 2] = 0.0
    sd = env.batch.state_dict()
    env.reset(noise)                          # wg_reset, in3d = 0: x, y only
    torch.cuda.synchronize()
    ref = env.vel.clone()
    env.batch.load_state_dict(sd)
    _lib.check(_lib.load().wg_reset_noise(C.byref(env.batch.struct), C.c_void_p(noise.data_ptr()),
                                          C.c_void_p(torch.cuda.current_stream().cuda_stream)), "wg_reset_noise")
    torch.cuda.synchronize()
    got = env.vel
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
    assert (got[:, 2].view(torch.int32) == np.int32(-2 ** 31)).all()   # still -0.0


def test_rollout_into_dirty_buffer_zero_pads():
    """A caller-supplied obs buffer is not assumed clean: the short rows' padding is written as zeros; the env's own
    (zero-initialised) buffers get only each row's own values (wg_outputs.obs_pad_clean)."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import ragged_walkers
    N, T = 300, 4
    spec = ragged_walkers(N, seed=12, mmin=3, mmax=30)
    A = int(np.max(spec["n_muscles"]))
    acts = np.random.default_rng(12).uniform(-1, 1, (T, N, A)).astype(np.float32)
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    sd = env.batch.state_dict()
    clean, _, _ = env.rollout(acts)
    env.batch.load_state_dict(sd)
    dirty = torch.full((T, N, env.obs_dim), 7.0, device="cuda:0")
    got, _, _ = env.rollout(acts, obs_out=dirty)
    torch.cuda.synchronize()
    assert torch.equal(got, clean)
    lens = env.obs_len
    for w in range(N):
        assert (clean[:, w, lens[w]:] == 0).all()


def test_plan_follows_params():
    """A uniform batch whose M does not divide 64 (M = 25) runs wave tiles for engine springs without pair forces,
    uniform workgroup tiles with pair forces; set_params re-plans both ways and every step stays bit-exact."""
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    N = 700
    spec = canonical_walkers(N, seed=61, M=25, K=60, A=10)
    acts = np.random.default_rng(61).uniform(-1, 1, (9, N, 10)).astype(np.float32)
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    orc = Oracle(spec, dict(in3d=1))
    kinds = []
    for t, pm in enumerate([0, 0, 0, 24, 24, 24, 0, 0, 0]):
        if pm != env.params.pair_mode:
            env.set_params(pair_mode=pm, pair_g=300.0)
            orc.set_params(pair_mode=pm, pair_g=300.0)
        kinds.append(env.batch.ragged_kind)
        obs, rew, done, info = env.step(acts[t])
        ref = orc.step(acts[t])
        torch.cuda.synchronize()
        assert np.array_equal(obs.cpu().numpy(), ref["obs"], equal_nan=True), t
    assert kinds == [2, 2, 2, 0, 0, 0, 2, 2, 2]
    assert np.array_equal(env.pos.cpu().numpy(), orc.pos, equal_nan=True)


def test_state_dict_independent_of_storage_order():
    """a ragged batch's storage order depends on WG_TILE_ORDER (read when the batch is packed); a state
    dict saved under one order loads into a batch stored in another and both continue bit-identically."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import ragged_walkers
    N = 900
    spec = ragged_walkers(N, seed=71, mmin=3, mmax=30)
    A = int(np.max(spec["n_muscles"]))
    acts = np.random.default_rng(71).uniform(-1, 1, (10, N, A)).astype(np.float32)
    os.environ["WG_TILE_ORDER"] = "sorted"
    try:
        a = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    finally:
        del os.environ["WG_TILE_ORDER"]
    b = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    assert not np.array_equal(a.batch.host.row, b.batch.host.row)
    a.rollout(acts[:5])
    b.batch.load_state_dict(a.batch.state_dict())
    oa, ra, _ = a.rollout(acts[5:])
    ob, rb, _ = b.rollout(acts[5:])
    torch.cuda.synchronize()
    assert torch.equal(oa, ob) and torch.equal(ra, rb)
    for k in ("pos", "vel", "acc", "muscle_x", "steps"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k


def test_state_setters_write_through_permuted_batch():
    """the state properties of a permuted (ragged) batch are gathered copies; assignment scatters the
    caller-order values into the stored order."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import ragged_walkers
    env = BatchedPhysicsEnv(ragged_walkers(300, seed=81, mmin=3, mmax=30), device="cuda:0", in3d=1)
    assert env.batch.row is not None
    for k in ("pos", "vel", "acc", "muscle_x"):
        want = torch.rand_like(getattr(env, k))
        setattr(env, k, want)
        assert torch.equal(getattr(env, k), want), k


def test_out_of_cap_wave_plan_is_skipped_and_reported():
    """wg_step trusts a device plan.  A wave-tile plan whose tiles exceed the wave caps (here: every
    walker in tile 0, empty tiles after it) must not write past the wave's LDS slice: the kernel skips such tiles
    (their walkers keep their state) and raises the flag wg_plan_errors reads."""
    import torch
    from walker_gym_amd import _lib
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import ragged_walkers
    L = _lib.load()
    spec = ragged_walkers(400, seed=91, mmin=4, mmax=30)
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    assert env.batch.ragged_kind == 2
    L.wg_plan_errors(1)
    A = int(np.max(spec["n_muscles"]))
    acts = torch.zeros((400, A), device="cuda:0")
    env.step(acts)                                   # a valid plan: no flag
    torch.cuda.synchronize()
    assert L.wg_plan_errors(0) == 0
    pos0 = env.pos.clone()
    env.batch.plan[1:] = 400                         # tile 0 = every walker, the other tiles empty
    env.step(acts)
    torch.cuda.synchronize()
    assert L.wg_plan_errors(1) == 1 and L.wg_plan_errors(0) == 0
    assert torch.equal(env.pos, pos0)


@pytest.mark.gpu
def test_info_steps_caller_order_without_gather():
    """A permuted (ragged) batch's info['steps'] comes from the kernels' caller-order steps output (wg_outputs.steps,
    ABI 9) after step() / run() / observe(), and from a gather after rollout() or loaded state: equal to the stored
    counters in the caller's order either way."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import ragged_walkers
    N = 700
    spec = ragged_walkers(N, seed=21, mmin=4, mmax=30)
    A = int(np.max(spec["n_muscles"]))
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    assert env.steps_out is not None
    acts = torch.rand((6, N, A), device="cuda:0") * 2 - 1

    def check(expect_out):
        info = env.info()
        torch.cuda.synchronize()
        ref = env.batch.caller("steps")
        assert torch.equal(info["steps"], ref)
        assert (info["steps"].data_ptr() == env.steps_out.data_ptr()) == expect_out
        return ref

    for t in range(3):
        env.step(acts[t])
    assert (check(True) == 3).all()
    env.run(acts[3:5].contiguous(), 2)
    assert (check(True) == 5).all()
    env.rollout(acts[:2])
    assert (check(False) == 7).all()
    mask = torch.zeros(N, dtype=torch.uint8, device="cuda:0")
    mask[::3] = 1
    env.reset(mask=mask)
    got = check(True)
    assert (got[::3] == 0).all() and (got[1::3] == 7).all()
    sd = env.batch.state_dict()
    env.step(acts[5])
    env.batch.load_state_dict(sd)
    assert torch.equal(check(False), got)
    # graph replay: after a step() (steps_out valid), a graph captured with info=False advances the
    # counters without writing steps_out, so info() must gather; one captured with info=True keeps steps_out current
    env.step(acts[0])
    check(True)
    g0 = env.graph(acts[1:3].contiguous(), 2, info=False)
    check(True)                          # capture runs nothing
    g0.replay()
    after = check(False)
    assert torch.equal(after, got + 3)
    g1 = env.graph(acts[1:3].contiguous(), 2, info=True)
    g1.replay()
    assert torch.equal(check(True), got + 5)


@pytest.mark.gpu
def test_tiny_and_subnormal_means_exact():
    """The wave kernel's per-walker means go through fdiv_count (an exact reciprocal product) except for |sum| <
    2^-100, which takes the IEEE division: walkers whose x coordinates are scaled to ~1e-36 (normal, tiny means) and
    ~1e-40 (subnormal coordinates and means) give the workgroup kernel's (IEEE) and the oracle's bits."""
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import ragged_walkers
    N = 400
    spec = ragged_walkers(N, seed=77, mmin=3, mmax=40)
    mo = spec["mass_off"]
    for w in range(N):
        spec["pos"][mo[w]:mo[w + 1], 0] *= np.float32(1e-36 if w % 2 else 1e-40)
    A = int(np.max(spec["n_muscles"]))
    acts = np.random.default_rng(77).uniform(-1, 1, (6, N, A)).astype(np.float32)
    env, wave = _rollout(spec, dict(in3d=1), acts, lean=True)
    assert env.batch.ragged_kind == 2
    _, wg = _rollout(spec, dict(in3d=1), acts, lean=False)
    for x, y in zip(wave, wg):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8))
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    orc = Oracle(spec, dict(in3d=1))
    for t in range(3):
        obs, rew, done, info = env.step(acts[t])
        ref = orc.step(acts[t])
    torch.cuda.synchronize()
    cen = info["centroid_position"].cpu().numpy()
    assert (np.abs(cen[:, 0]) < 1e-30).all() and (np.abs(cen[0::2, 0]) < 1.2e-38).any()   # subnormal means reached
    assert np.array_equal(cen.view(np.uint32), ref["centroid"].view(np.uint32))
    assert np.array_equal(obs.cpu().numpy().view(np.uint32), ref["obs"].view(np.uint32))


def test_full_size_ragged_vs_oracle():
    """BASELINE config 5 at its full size (65,536 walkers, M ~ U{4..32}, the bench's batch: wave tiles in best-fit
    windowed order, XCD-aware), every walker (the round-4 test compared a sample of 516): 8 full-batch GPU
    steps against the C oracle stepping the same batch in the caller's order — positions, velocities, observations
    with their zero padding, reward, done, centroid, energy, bit for bit."""
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import ragged_walkers
    N, T = 65536, 8
    spec = ragged_walkers(N, seed=0, mmin=4, mmax=32)
    A = int(np.max(spec["n_muscles"]))
    rng = np.random.default_rng(3)
    acts = rng.uniform(-1, 1, (T, N, A)).astype(np.float32)
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    assert env.batch.ragged_kind == 2
    orc = Oracle(spec, dict(in3d=1), n_threads=16)
    for t in range(T):
        obs, rew, done, info = env.step(acts[t])
        ref = orc.step(acts[t])
    torch.cuda.synchronize()
    assert np.array_equal(env.pos.cpu().numpy().view(np.uint32), orc.pos.view(np.uint32))
    assert np.array_equal(env.vel.cpu().numpy().view(np.uint32), orc.vel.view(np.uint32))
    o = obs.cpu().numpy()
    D = ref["obs"].shape[1]
    assert np.array_equal(o[:, :D].view(np.uint32), ref["obs"].view(np.uint32)) and not o[:, D:].any()
    assert np.array_equal(rew.cpu().numpy().view(np.uint32), ref["reward"].view(np.uint32))
    assert np.array_equal(done.cpu().numpy(), ref["done"])
    assert np.array_equal(info["centroid_position"].cpu().numpy().view(np.uint32), ref["centroid"].view(np.uint32))
    assert np.array_equal(info["total_energy"].cpu().numpy().view(np.uint32), ref["energy"].view(np.uint32))
