"""GPU parity: the HIP path (through the C ABI) against the reference goldens and the CPU oracle.

Contract (BASELINE.json north_star: "match the reference CPU engine ... to a stated fp32 tolerance"):
  pos / vel / acc / muscle x / obs / reward / centroid within atol = 1e-4, rtol = 1e-5
  over <= 100 steps; contact / done / steps exactly.  energy bit-exact: numpy's float32 ``** 2`` is libm
  powf (not x*x), which the kernel restates (walker_gym_amd/csrc/powf2.h, pinned exhaustively on the host).
What is asserted is stronger than that contract: the kernel restates numpy's arithmetic op by op, and every float
field must be BIT-identical to the reference fixtures and to the oracle (``_close`` checks the tolerance first, so a
regression reports against the contract, then the bits; NaN payloads excepted).  ``test_bit_exact_fraction`` counts
the identical elements over every golden step, requires all of them, and reports the fraction in the session
summary (conftest.record_metric).
"""
import glob
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))
ATOL, RTOL = 1e-4, 1e-5


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no ROCm GPU")


def _env_from_npz(z, **over):
    from oracle.oracle import spec_from_npz
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    spec, params = spec_from_npz(z)
    params.update(over)
    env = BatchedPhysicsEnv(spec, **{k: v for k, v in params.items()})
    return env, spec, params


def _bits_equal(got, ref):
    """Elementwise bit identity of two float32 arrays (+0.0 and -0.0 differ); NaN == NaN whatever the payload."""
    g = np.ascontiguousarray(np.asarray(got, np.float32).reshape(ref.shape))
    r = np.ascontiguousarray(np.asarray(ref, np.float32))
    return (g.view(np.uint32) == r.view(np.uint32)) | (np.isnan(g) & np.isnan(r))


def _close(got, ref, atol=ATOL, rtol=RTOL):
    raw = got
    got = np.asarray(got, np.float64).reshape(ref.shape)
    ref64 = ref.astype(np.float64)
    fin = np.isfinite(ref64)
    assert np.array_equal(np.isfinite(got), fin), "non-finite pattern differs"
    assert np.array_equal(np.isnan(got), np.isnan(ref64)), "NaN pattern differs"
    if fin.any():
        np.testing.assert_allclose(got[fin], ref64[fin], atol=atol, rtol=rtol)   # the stated contract
    inf = np.isinf(ref64)
    assert np.array_equal(got[inf], ref64[inf])
    if ref.dtype == np.float32:   # the product's claim: bit-identical
        eq = _bits_equal(raw, ref)
        assert eq.all(), f"{int((~eq).sum())} of {eq.size} elements within tolerance but not bit-identical"


def _run_golden(path):
    import torch
    z = np.load(path)
    env, spec, params = _env_from_npz(z)
    noise = z["noise"] if z["noise"].size else None
    obs0 = (env.reset(noise) if noise is not None else env.observe()[0]).clone()
    steps = []
    for t in range(z["out_pos"].shape[0]):
        a = z["actions"][t] if z["actions"].shape[2] else None
        obs, rew, done, info = env.step(a)
        torch.cuda.synchronize()
        steps.append(dict(pos=env.pos.cpu().numpy(), vel=env.vel.cpu().numpy(), acc=env.acc.cpu().numpy(),
                          mx=env.muscle_x.cpu().numpy(), contact=env.contact.cpu().numpy(),
                          obs=obs.cpu().numpy(), reward=rew.cpu().numpy(), done=done.cpu().numpy().astype(np.uint8),
                          centroid=info["centroid_position"].cpu().numpy(), energy=info["total_energy"].cpu().numpy(),
                          steps=info["steps"].cpu().numpy()))
    return z, obs0.cpu().numpy(), steps


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[:-4] for f in FILES])
def test_gpu_matches_reference_golden(path):
    z, obs0, steps = _run_golden(path)
    _close(obs0, z["out_obs0"])
    for t, got in enumerate(steps):
        for f in ("pos", "vel", "acc", "mx", "obs", "reward", "centroid"):
            _close(got[f], z["out_" + f][t])
        for f in ("contact", "done", "steps"):
            assert np.array_equal(got[f].reshape(z["out_" + f][t].shape), z["out_" + f][t]), (t, f)
        e = np.asarray(got["energy"]).reshape(z["out_energy"][t].shape)
        assert np.array_equal(e, z["out_energy"][t], equal_nan=True), (t, "energy")


def test_bit_exact_fraction():
    """Every float field of every golden step bit-identical to the reference (signed zeros included): fraction 1.0."""
    from conftest import record_metric
    tot = same = 0
    for path in FILES:
        z, obs0, steps = _run_golden(path)
        for t, got in enumerate(steps):
            for f in ("pos", "vel", "acc", "mx", "obs", "reward", "centroid", "energy"):
                ref = z["out_" + f][t]
                eq = _bits_equal(got[f], ref)
                tot += eq.size
                same += int(eq.sum())
    frac = same / tot
    record_metric("bit_exact_fraction_vs_reference", f"{frac:.9f} ({same} of {tot} float elements over "
                                                     f"{len(FILES)} golden files; {tot - same} differ)")
    assert same == tot, f"{tot - same} of {tot} elements differ from the reference bits"


def _oracle_compare(spec, params, T, actions, rtol=RTOL, atol=ATOL):
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    env = BatchedPhysicsEnv(spec, **params)
    orc = Oracle(spec, params, n_threads=8)
    for t in range(T):
        a = actions[t]
        obs, rew, done, info = env.step(a)
        ref = orc.step(a)
        torch.cuda.synchronize()
        _close(env.pos.cpu().numpy(), orc.pos, atol, rtol)
        _close(env.vel.cpu().numpy(), orc.vel, atol, rtol)
        _close(obs.cpu().numpy(), ref["obs"], atol, rtol)
        _close(rew.cpu().numpy(), ref["reward"], atol, rtol)
        assert np.array_equal(done.cpu().numpy().astype(np.uint8), ref["done"])
        assert np.array_equal(env.contact.cpu().numpy(), orc.contact)
    return env, orc


def test_canonical_4096_vs_oracle():
    from walker_gym_amd.synthetic import canonical_walkers
    spec = canonical_walkers(4096, seed=1)
    acts = np.random.default_rng(1).uniform(-1, 1, (30, 4096, 8)).astype(np.float32)
    _oracle_compare(spec, dict(in3d=1), 30, acts)


def test_balance_4096_vs_oracle():
    """BASELINE config 2: 4,096 identical Balance-v0 walkers."""
    from walker_gym_amd.walker import balance_spec
    spec = balance_spec(4096)
    acts = np.random.default_rng(2).uniform(-1, 1, (50, 4096, 2)).astype(np.float32)
    _oracle_compare(spec, dict(in3d=0), 50, acts)


def test_ragged_2000_vs_oracle():
    """BASELINE config 5: mixed topologies through the ragged (planned) path."""
    from walker_gym_amd.synthetic import ragged_walkers
    spec = ragged_walkers(2000, seed=3, mmin=2, mmax=40, string_frac=0.1)
    A = int(np.max(spec["n_muscles"]))
    acts = np.random.default_rng(3).uniform(-1, 1, (20, 2000, A)).astype(np.float32)
    _oracle_compare(spec, dict(in3d=1, dampk=0.3), 20, acts)


def test_imported_topologies_vs_oracle():
    """G1 builders (M=4 creatures take the lean kernel, observed with G1 getstat,
    midform 2) and a ragged batch of every G3 builder (pinned m=0 pivots included)."""
    from walker_gym_amd.topologies import G3_BUILDERS, mixed_spec, topology_spec
    rng = np.random.default_rng(9)
    cases = ((topology_spec("box2", 997, 1), dict(in3d=0, midform=2, conmid=1)),
             (topology_spec("insect", 500, 1), dict(in3d=0, midform=2)),
             (mixed_spec([(n, 40) for n in G3_BUILDERS], 3), dict(in3d=1, ground=-30.0)))
    for spec, params in cases:
        N = len(spec["mass_off"]) - 1
        A = max(1, int(np.max(spec["n_muscles"])))
        acts = rng.uniform(-1, 1, (20, N, A)).astype(np.float32)
        _oracle_compare(spec, params, 20, acts)


@pytest.mark.parametrize("pair_mode", [7, 24, 31, "4_subset", "31_subset"])
def test_pair_forces_4096_vs_oracle(pair_mode):
    """pair_mode bits in order (gravity, coulomb, bounce of gym/engine.py:114-147; 8 G2 gravity_vec,
    gym/optimized_engine.py:167-197; 16 electrostatic, gym/engine.py:150-158), per walker on the lean kernel, on 4096
    shrunk canonical walkers with per-mass charges and radii: bit-exact positions/velocities and the env-updated
    radii."""
    import torch
    from walker_gym_amd.synthetic import canonical_walkers
    N = 4096
    spec = canonical_walkers(N, seed=5)
    spec["pos"] = (spec["pos"] * np.float32(0.4)).astype(np.float32)
    spec["rest"] = (spec["rest"] * np.float32(0.4)).astype(np.float32)
    rng = np.random.default_rng(5)
    spec["charge"] = rng.uniform(-3, 3, 16 * N)
    spec["radius"] = rng.uniform(1.5, 3.0, 16 * N)
    if isinstance(pair_mode, str):   # Point.bounce(k, other=<list>): random caller / list bits (wg_batch.bounce_set)
        pair_mode = int(pair_mode.split("_")[0])
        spec["bounce_set"] = rng.integers(0, 4, 16 * N).astype(np.uint8)
    params = dict(in3d=1, pair_mode=pair_mode, pair_g=2000.0, pair_k=1.0e4, bounce_k=2000.0)
    acts = rng.uniform(-1, 1, (20, N, 8)).astype(np.float32)
    env, orc = _oracle_compare(spec, params, 20, acts, rtol=0, atol=0)
    torch.cuda.synchronize()
    if pair_mode & 4:
        assert np.array_equal(env.batch.radius.cpu().numpy(), orc.radius)
    # close opposite charges blow ~1 % of the walkers up to inf/NaN, in the reference's arithmetic too
    assert np.array_equal(env.pos.cpu().numpy(), orc.pos, equal_nan=True)
    assert np.isfinite(orc.pos).all(1).mean() > 0.95


@pytest.mark.parametrize("case", ["M64_K160", "M4_K6", "M16_partial_tile", "M64_K300_NE5", "ragged_M256"])
def test_size_extremes_vs_oracle(case):
    """Edges of the launch geometry against the oracle: the largest lean tile (M = 64, one walker per wave,
    3 and 5 edge passes), the smallest (M = 4, 16 walkers per wave), a batch that ends mid-wave, and ragged
    walkers up to M = 256 on the workgroup kernel."""
    from walker_gym_amd.synthetic import canonical_walkers, ragged_walkers
    if case == "M64_K160":
        spec, A, N = canonical_walkers(96, seed=11, M=64, K=160, A=20), 20, 96
    elif case == "M64_K300_NE5":
        spec, A, N = canonical_walkers(64, seed=12, M=64, K=300, A=8), 8, 64
    elif case == "M4_K6":
        spec, A, N = canonical_walkers(1000, seed=13, M=4, K=6, A=2), 2, 1000
    elif case == "M16_partial_tile":
        spec, A, N = canonical_walkers(4097, seed=14), 8, 4097
    else:
        spec = ragged_walkers(300, seed=15, mmin=100, mmax=256, string_frac=0.1)
        N, A = 300, int(np.max(spec["n_muscles"]))
    acts = np.random.default_rng(11).uniform(-1, 1, (8, N, A)).astype(np.float32)
    _oracle_compare(spec, dict(in3d=1), 8, acts)


def test_uniform_non_divisor_M_on_wave_kernel():
    """A uniform batch whose M does not divide 64 (5x5 lattice, M = 25) is stepped as wave tiles of whole walkers
    (the barrier-free wave kernel, identity order): oracle parity, and bitwise equal to the workgroup kernel
    (WG_UNIFORM_WAVES=0, read when the device batch is built)."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    N = 3000
    spec = canonical_walkers(N, seed=31, M=25, K=60, A=10)
    acts = np.random.default_rng(31).uniform(-1, 1, (12, N, 10)).astype(np.float32)
    env, _ = _oracle_compare(spec, dict(in3d=1), 12, acts)
    assert env.batch.ragged_kind == 2 and env.batch.row is None
    outs = []
    for flag in ("1", "0"):
        os.environ["WG_UNIFORM_WAVES"] = flag
        try:
            e = BatchedPhysicsEnv(spec, in3d=1)
        finally:
            del os.environ["WG_UNIFORM_WAVES"]
        assert e.batch.ragged_kind == (2 if flag == "1" else 0)
        o, r, d = e.rollout(acts, resident=False)
        torch.cuda.synchronize()
        outs.append([o.cpu().numpy(), r.cpu().numpy(), e.pos.cpu().numpy(), e.vel.cpu().numpy()])
    for x, y in zip(*outs):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8))


def _tiny_walkers(N, seed):
    """Walkers of 1-3 masses: single free masses (no spring), pairs with one spring, triangles; some with no
    muscle.  Exercises the smallest tiles of the workgroup kernel."""
    rng = np.random.default_rng(seed)
    m, pos, mo, ei, ej, rest, eo, nm = [], [], [0], [], [], [], [0], []
    for w in range(N):
        M = int(rng.integers(1, 4))
        p = rng.uniform(-5, 5, (M, 3)).astype(np.float32)
        p[:, 1] += 3.0
        m += list(rng.uniform(0.5, 3, M)); pos += list(p); mo.append(mo[-1] + M)
        pairs = [(0, 1)] if M == 2 else ([(0, 1), (1, 2), (0, 2)] if M == 3 else [])
        for i, j in pairs:
            ei.append(i); ej.append(j); rest.append(float(np.linalg.norm(p[i] - p[j])) * 0.9)
        eo.append(len(ei))
        nm.append(min(len(pairs), int(rng.integers(0, 2))))
    E, U = len(ei), int(sum(nm))
    P = len(m)
    return dict(m=np.array(m, np.float32), pos=np.array(pos, np.float32), vel=np.zeros((P, 3), np.float32),
                mass_off=np.array(mo, np.int32), ei=np.array(ei, np.int32), ej=np.array(ej, np.int32),
                rest=np.array(rest, np.float32), k=np.full(E, 500.0, np.float32), c=np.full(E, 10.0, np.float32),
                flags=(rng.random(E) < 0.3).astype(np.uint8), edge_off=np.array(eo, np.int32),
                n_muscles=np.array(nm, np.int32), minl=np.full(U, 0.5, np.float32),
                maxl=np.full(U, 1.5, np.float32), stride=np.full(U, 1.0, np.float32))


def test_tiny_walkers_vs_oracle():
    spec = _tiny_walkers(3000, seed=21)
    acts = np.random.default_rng(21).uniform(-1, 1, (30, 3000, 1)).astype(np.float32)
    _oracle_compare(spec, dict(in3d=1), 30, acts)


def _big_walkers(N, M, K, A, seed):
    """N walkers of M masses and K random springs (the first A muscles)."""
    from walker_gym_amd.synthetic import norm3_f32
    rng = np.random.default_rng(seed)
    pos = rng.uniform(-20, 20, (N * M, 3)).astype(np.float32)
    pos[:, 1] += 25.0
    ei = rng.integers(0, M, N * K).astype(np.int32)
    ej = ((ei + rng.integers(1, M, N * K)) % M).astype(np.int32)
    base = np.repeat(np.arange(N) * M, K)
    rest = norm3_f32(pos[base + ei] - pos[base + ej]).astype(np.float32)
    return dict(m=rng.uniform(1, 3, N * M).astype(np.float32), pos=pos, vel=np.zeros((N * M, 3), np.float32),
                mass_off=(np.arange(N + 1) * M).astype(np.int32), ei=ei, ej=ej, rest=rest,
                k=np.full(N * K, 200.0, np.float32), c=np.full(N * K, 5.0, np.float32),
                flags=np.zeros(N * K, np.uint8), edge_off=(np.arange(N + 1) * K).astype(np.int32),
                n_muscles=np.full(N, A, np.int32), minl=np.full(N * A, 0.5, np.float32),
                maxl=np.full(N * A, 1.5, np.float32), stride=np.full(N * A, 1.0, np.float32))


def test_largest_walkers():
    """WG_MAX_M = 1024 masses: 1024-mass, 1024-spring walkers match the oracle on the workgroup kernel; walkers
    whose spring terms cannot fit a workgroup's 160 KiB of LDS are refused before any launch (WG_ERANGE)."""
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    spec = _big_walkers(3, 1024, 1024, 8, seed=31)
    acts = np.random.default_rng(31).uniform(-1, 1, (4, 3, 8)).astype(np.float32)
    _oracle_compare(spec, dict(in3d=1), 4, acts)
    with pytest.raises(ValueError, match="LDS"):
        BatchedPhysicsEnv(_big_walkers(2, 1024, 6000, 0, seed=32), in3d=1).step(None)


def test_from_topologies_vs_oracle():
    """BatchedPhysicsEnv.from_topologies: 4000 envs over Balance-v0 and Box-v0 vs the oracle."""
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.walker import (concat_specs, create_balance_creature, create_box_creature,
                                       creatures_to_spec, replicate_spec)
    env = BatchedPhysicsEnv.from_topologies(["Balance-v0", "Box-v0"], 4000, device="cuda:0", in3d=1)
    spec = concat_specs([replicate_spec(creatures_to_spec([create_balance_creature()]), 2000),
                         replicate_spec(creatures_to_spec([create_box_creature()]), 2000)])
    orc = Oracle(spec, dict(in3d=1))
    acts = np.random.default_rng(8).uniform(-1, 1, (20, 4000, 4)).astype(np.float32)
    for t in range(20):
        obs, rew, done, info = env.step(acts[t])
        ref = orc.step(acts[t])
    torch.cuda.synchronize()
    _close(env.pos.cpu().numpy(), orc.pos)
    _close(obs.cpu().numpy(), ref["obs"])
    with pytest.raises(ValueError, match="Unknown environment ID"):
        BatchedPhysicsEnv.from_topologies("Walker-v9", 8, device="cuda:0")


def test_reset_noise_entry_point():
    """wg_reset_noise == PhysicsEnv.reset with all three noise components (wg_reset, in3d)."""
    import ctypes as C

    import torch
    from walker_gym_amd import _lib
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    N = 2048
    env = BatchedPhysicsEnv(canonical_walkers(N, seed=17), device="cuda:0", in3d=1)
    acts = np.random.default_rng(17).uniform(-1, 1, (5, N, 8)).astype(np.float32)
    for t in range(5):
        env.step(acts[t])
    sd = env.batch.state_dict()
    noise = torch.randn((N * 16, 3), generator=torch.Generator(device="cuda:0").manual_seed(17), device="cuda:0")
    env.reset(noise)
    torch.cuda.synchronize()
    ref = [t.clone() for t in env.batch.state_dict().values()]
    env.batch.load_state_dict(sd)
    _lib.check(_lib.load().wg_reset_noise(C.byref(env.batch.struct), C.c_void_p(noise.data_ptr()),
                                          C.c_void_p(torch.cuda.current_stream().cuda_stream)), "wg_reset_noise")
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(ref, env.batch.state_dict().values()))


def test_full_size_vs_oracle():
    """BASELINE config 3 at its full size (65,536 canonical walkers), every walker (the round-4 test compared a
    sample of 512): 10 full-batch GPU steps against the C oracle stepping the same batch (OpenMP over walkers), every
    state and output field bit for bit."""
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    N, T = 65536, 10
    spec = canonical_walkers(N, seed=0)
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (T, N, 8)).astype(np.float32)
    env = BatchedPhysicsEnv(spec, in3d=1)
    orc = Oracle(spec, dict(in3d=1), n_threads=16)
    for t in range(T):
        obs, rew, done, info = env.step(acts[t])
        out = orc.step(acts[t])
    torch.cuda.synchronize()
    _close(env.pos.cpu().numpy(), orc.pos)
    _close(env.vel.cpu().numpy(), orc.vel)
    _close(env.acc.cpu().numpy(), orc.acc)
    _close(obs.cpu().numpy(), out["obs"])
    _close(rew.cpu().numpy(), out["reward"])
    assert np.array_equal(done.cpu().numpy(), out["done"])
    _close(info["centroid_position"].cpu().numpy(), out["centroid"])
    _close(info["total_energy"].cpu().numpy(), out["energy"])


def _subset(spec, idx):
    """Uniform spec restricted to walkers idx."""
    N = len(spec["mass_off"]) - 1
    M = int(spec["mass_off"][1]); K = int(spec["edge_off"][1]); A = int(spec["n_muscles"][0])
    n = len(idx)
    out = dict(spec)
    for key, per in (("m", M), ("pos", M), ("vel", M), ("acc", M), ("ei", K), ("ej", K), ("rest", K), ("k", K),
                     ("c", K), ("flags", K), ("minl", A), ("maxl", A), ("stride", A)):
        arr = np.asarray(spec[key])
        out[key] = arr.reshape((N, per) + arr.shape[1:])[idx].reshape((n * per,) + arr.shape[1:])
    out["mass_off"] = (np.arange(n + 1) * M).astype(np.int32)
    out["edge_off"] = (np.arange(n + 1) * K).astype(np.int32)
    out["n_muscles"] = np.full(n, A, np.int32)
    return out


def test_determinism_and_shard_equivalence():
    """Two runs are bitwise identical, and a shard run alone equals the same walkers in the full
    batch (what makes the multi-GPU weak-scaling path exact)."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    N = 8192
    spec = canonical_walkers(N, seed=5)
    acts = np.random.default_rng(5).uniform(-1, 1, (20, N, 8)).astype(np.float32)
    runs = []
    for _ in range(2):
        env = BatchedPhysicsEnv(spec, in3d=1)
        o, r, d = env.rollout(acts)
        torch.cuda.synchronize()
        runs.append((env.pos.cpu().numpy(), o.cpu().numpy(), r.cpu().numpy()))
    for a, b in zip(runs[0], runs[1]):
        assert np.array_equal(a, b)
    half = np.arange(N // 2, N)
    env = BatchedPhysicsEnv(_subset(spec, half), in3d=1)
    o, r, d = env.rollout(acts[:, half])
    torch.cuda.synchronize()
    assert np.array_equal(env.pos.cpu().numpy(), runs[0][0].reshape(N, 16, 3)[half].reshape(-1, 3))
    assert np.array_equal(o.cpu().numpy(), runs[0][1][:, half])


def test_rollout_equals_stepwise():
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    spec = canonical_walkers(1000, seed=8)
    acts = np.random.default_rng(8).uniform(-1, 1, (15, 1000, 8)).astype(np.float32)
    e1 = BatchedPhysicsEnv(spec, in3d=1)
    o, r, d = e1.rollout(acts)
    e2 = BatchedPhysicsEnv(spec, in3d=1)
    for t in range(15):
        ob, rw, dn, _ = e2.step(acts[t])
        torch.cuda.synchronize()
        assert np.array_equal(ob.cpu().numpy(), o[t].cpu().numpy())
        assert np.array_equal(rw.cpu().numpy(), r[t].cpu().numpy())


@pytest.mark.parametrize("case", ["canonical", "balance2d_discrete", "run2_pinned", "canonical_long_lanes2"])
def test_resident_rollout_bit_identical(case):
    """wg_rollout (one launch, state in registers across steps) == wg_step per step: every step's obs / reward /
    done and the final state (pos, vel, acc, muscle x, steps, contact), bit for bit."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    from walker_gym_amd.walker import create_balance_creature, creatures_to_spec, replicate_spec
    T, lanes, params = 25, 1, dict(in3d=1)
    if case.startswith("canonical"):
        N = 3000 if case == "canonical" else 20000
        spec = canonical_walkers(N, seed=11)
        if case == "canonical_long_lanes2":
            T, lanes = 130, 2          # past steps > 100: the all-stopped done branch is live
    elif case == "balance2d_discrete":
        N = 5000
        spec = replicate_spec(creatures_to_spec([create_balance_creature()]), N)
        params = dict(in3d=0, action_mode=1)
    else:
        N = 4096
        spec = canonical_walkers(N, seed=12)
        spec["pinned"] = (np.random.default_rng(12).random(len(spec["m"])) < 0.05).astype(np.uint8)
        params = dict(in3d=1, integrator=2)
    A = int(spec["n_muscles"].max())
    acts = np.random.default_rng(13).uniform(-1, 1, (T, N, A)).astype(np.float32)
    if params.get("action_mode") == 1:
        acts = np.where(acts > 0, 1.0, 0.0).astype(np.float32)
    got = []
    for resident in (False, True):
        env = BatchedPhysicsEnv(spec, **params)
        o, r, d = env.rollout(acts, lanes=lanes, resident=resident)
        torch.cuda.synchronize()
        st = env.batch.state_dict()
        got.append([o.cpu(), r.cpu(), d.cpu()] + [t.cpu() for t in st.values()])
    assert len(got[0]) == len(got[1])
    for k, (a, b) in enumerate(zip(*got)):   # NaN == NaN: a walker that blows up does so on both paths
        assert np.array_equal(a.numpy(), b.numpy(), equal_nan=a.dtype.is_floating_point), (case, k)


def test_run_lanes_bit_identical(monkeypatch):
    """run() with the walkers split over 2 / 3 streams (lanes) gives the same bits as one stream, with the ranges
    issued step by step (wg_run_ranges, the default) and range by range (WG_RANGE_ISSUE=seq)."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    N = 10000
    env = BatchedPhysicsEnv(canonical_walkers(N, seed=3), device="cuda:0", in3d=1)
    acts = (torch.rand((40, N, 8), generator=torch.Generator(device="cuda:0").manual_seed(3), device="cuda:0")
            * 2 - 1).contiguous()
    sd0 = env.batch.state_dict()
    ref = None
    for lanes, issue in ((1, "inter"), (2, "inter"), (3, "inter"), (2, "seq")):
        monkeypatch.setenv("WG_RANGE_ISSUE", issue)
        env.batch.load_state_dict(sd0)
        env.run(acts, 40, lanes=lanes)
        torch.cuda.synchronize()
        got = [t.clone() for t in env.batch.state_dict().values()] + [env.obs.clone(), env.reward.clone(),
                                                                       env.done.clone(), env.energy.clone()]
        if ref is None:
            ref = got
        else:
            assert all(torch.equal(a, b) for a, b in zip(ref, got)), lanes
    # ragged batch: ranges of plan blocks
    from walker_gym_amd.synthetic import ragged_walkers
    rg = BatchedPhysicsEnv(ragged_walkers(20000, seed=4, string_frac=0.2), device="cuda:0", in3d=1)
    assert rg._lanes(2) == 2, rg.batch.plan_blocks
    ra = (torch.rand((20, 20000, int(rg.batch.A)), generator=torch.Generator(device="cuda:0").manual_seed(4),
                     device="cuda:0") * 2 - 1).contiguous()
    rsd = rg.batch.state_dict()
    rres = []
    for lanes, issue in ((1, "inter"), (2, "inter"), (2, "seq")):
        monkeypatch.setenv("WG_RANGE_ISSUE", issue)
        rg.batch.load_state_dict(rsd)
        rg.run(ra, 20, lanes=lanes)
        torch.cuda.synchronize()
        rres.append([t.clone() for t in rg.batch.state_dict().values()] + [rg.obs.clone(), rg.reward.clone()])
    assert all(torch.equal(a, b) for a, b in zip(rres[0], rres[1])) and all(torch.equal(a, b) for a, b in zip(rres[0], rres[2]))
    monkeypatch.setenv("WG_RANGE_ISSUE", "inter")
    # rollout(): per-step outputs of every range land in the right rows
    outs = []
    for lanes in (1, 2):
        env.batch.load_state_dict(sd0)
        outs.append([t.clone() for t in env.rollout(acts[:12], lanes=lanes)])
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(*outs))


@pytest.mark.parametrize("kind,lanes", [("canonical", 2), ("ragged", 2), ("canonical", 3), ("ragged", 1)])
def test_graph_replay_equals_run(kind, lanes):
    """run() captured as HIP graphs (one per walker range, each replayed on its own stream) and replayed gives the
    same bits as the direct calls, uniform and ragged (plan slices) batches."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers, ragged_walkers
    N = 12000
    spec = canonical_walkers(N, seed=6) if kind == "canonical" else ragged_walkers(N, seed=6, mmin=4, mmax=32)
    env = BatchedPhysicsEnv(spec, device="cuda:0", in3d=1)
    A = env.batch.A
    acts = (torch.rand((10, N, A), generator=torch.Generator(device="cuda:0").manual_seed(6), device="cuda:0")
            * 2 - 1).contiguous()
    sd0 = env.batch.state_dict()
    env.run(acts, 10, lanes=1)
    env.run(acts, 10, lanes=1)
    torch.cuda.synchronize()
    ref = [t.clone() for t in env.batch.state_dict().values()] + [env.obs.clone(), env.energy.clone()]
    env.batch.load_state_dict(sd0)
    torch.cuda.synchronize()
    g = env.graph(acts, 10, lanes=lanes)   # capture records the launches (one graph per range) without running them
    env.batch.load_state_dict(sd0)
    torch.cuda.synchronize()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    got = [t.clone() for t in env.batch.state_dict().values()] + [env.obs.clone(), env.energy.clone()]
    assert all(torch.equal(a, b) for a, b in zip(ref, got))
    assert torch.equal(env.info()["steps"], torch.full((N,), 20, dtype=torch.int32, device="cuda:0"))
    # the graph holds the parameters and buffers as captured: after set_params it refuses to replay
    env.set_params(dampk=0.5)
    with pytest.raises(RuntimeError, match="stale"):
        g.replay()


def test_run_and_rollout_refuse_foreign_tensors():
    """run()/rollout() hand raw pointers to the kernel: host tensors, other dtypes and non-contiguous outputs are
    refused before any launch."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    env = BatchedPhysicsEnv(canonical_walkers(64, seed=1), device="cuda:0", in3d=1)
    good = torch.zeros((2, 64, 8), device="cuda:0")
    for bad in (torch.zeros((2, 64, 8)), torch.zeros((2, 64, 8), device="cuda:0", dtype=torch.float64),
                torch.zeros((2, 8, 64), device="cuda:0").transpose(1, 2)):
        with pytest.raises(ValueError):
            env.run(bad, 2)
    env.run(good, 2)
    with pytest.raises(ValueError):
        env.rollout(good, obs_out=torch.zeros((2, 64, env.obs_dim)))
    with pytest.raises(ValueError):
        env.rollout(good, done_out=torch.zeros((2, 64), device="cuda:0"))
    with pytest.raises(ValueError):
        env.rollout(good, reward_out=torch.zeros((64, 2), device="cuda:0").t())


def _variant_cases():
    from walker_gym_amd.synthetic import canonical_walkers
    from walker_gym_amd.topologies import topology_spec
    from walker_gym_amd.walker import balance_spec
    pinned = canonical_walkers(700, seed=13)
    pinned["pinned"] = (np.random.default_rng(13).random(700 * 16) < 0.1).astype(np.uint8)
    pinned["vel"] = np.random.default_rng(14).normal(0, 1, (700 * 16, 3)).astype(np.float32)
    return [("canonical", canonical_walkers(1003, seed=11), dict(in3d=1), 8),   # 1003: a partial last wave
            ("balance", balance_spec(997), dict(in3d=0), 2),
            ("canonical2d", canonical_walkers(640, seed=12), dict(in3d=0, dampk=0.2, midform=0), 8),
            ("pinned_run2", pinned, dict(in3d=1, integrator=2), 8),
            ("g1_box2", topology_spec("box2", 997, 1), dict(in3d=0, midform=2, conmid=1), 4)]


def _variant_run(spec, params, A, name):
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    N = len(spec["mass_off"]) - 1
    acts = np.random.default_rng(len(name)).uniform(-1, 1, (25, N, A)).astype(np.float32)
    env = BatchedPhysicsEnv(spec, device="cuda", **params)
    o, r, d = env.rollout(acts)
    torch.cuda.synchronize()
    out = [o, r, d] + [getattr(env, f)
                       for f in ("pos", "vel", "acc", "muscle_x", "contact", "steps")]
    return [t.cpu().numpy() for t in out]


def test_kernel_variants_agree():
    """The wave-independent lean kernel (default for uniform M | 64 batches) and the workgroup kernel
    (WG_LEAN=0, read by libwalker_hip.so on every call) restate the same arithmetic: their outputs must be
    bitwise equal, including a batch whose last wave is only partly filled."""
    for name, spec, params, A in _variant_cases():
        lean = _variant_run(spec, params, A, name)
        os.environ["WG_LEAN"] = "0"
        try:
            wg = _variant_run(spec, params, A, name)
        finally:
            del os.environ["WG_LEAN"]
        for x, y in zip(lean, wg):
            assert x.shape == y.shape, name
            assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), name


def test_launch_floor_probe():
    """wg_launch_floor (bench.py's same-box floor for small batches): mode 1 writes in + 1 over the whole grid, mode 0
    touches nothing, and bad arguments are refused."""
    import ctypes as C
    import torch
    from walker_gym_amd import _lib
    L = _lib.load()
    blocks, threads = 37, 256
    src = torch.arange(blocks * threads, dtype=torch.float32, device="cuda:0")
    dst = torch.full_like(src, -7.0)
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()))
    assert L.wg_launch_floor(0, blocks, threads, *args, 3, sp) == 0
    torch.cuda.synchronize()
    assert (dst == -7.0).all()
    assert L.wg_launch_floor(1, blocks, threads, *args, 2, sp) == 0
    torch.cuda.synchronize()
    assert torch.equal(dst, src + 1)
    assert L.wg_launch_floor(2, blocks, threads, *args, 2, sp) == 0   # the busy kernel (bench.py's device warm-up)
    assert L.wg_launch_floor(3, blocks, threads, *args, 1, sp) == _lib.WG_EINVAL
    assert L.wg_launch_floor(1, blocks, 2048, *args, 1, sp) == _lib.WG_EINVAL
