"""Diverged walkers (round 6): a walker every mass of which has a NaN position component (not pinned, with a spring)
steps on the kernels' stand-in path — its state, outputs and per-walker sums set to the NaN the reference computes —
while a walker only partly NaN, or with infinities, pinned masses or pair forces, steps exactly as before.  Everything
against the C oracle (the reference restated; pinned to the reference's own fixtures, two of which diverge: box 3D at
step 38 and info_extras at step 27), bit for bit with NaN == NaN whatever the payload, on the lean kernel (canonical
NE = 3, Balance-v0 2D NE = 1), the wave kernel (mixed topology) and the workgroup kernel (M = 25 without the wave
plan), plus the resident rollout (the stand-in path in its NE = 1 instance only) against per-step launches."""
import numpy as np
import pytest

from conftest import gpu_available
from test_gpu_parity import _close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no ROCm GPU")


def _diverge(spec, rng, n_dead=40, n_partial=20, n_inf=10, pin=True):
    """Inject divergence into walkers of a flat spec: dead walkers (a NaN component in every mass, the component and the
    velocity varying), partly NaN walkers, walkers at +inf, and dead walkers with one pinned mass (which therefore
    step exactly)."""
    mo = np.asarray(spec["mass_off"])
    N = len(mo) - 1
    pos, vel = spec["pos"].copy(), spec["vel"].copy()
    pinned = np.zeros(len(pos), np.uint8)
    w = rng.permutation(N)
    dead, part, inf, pinw = (w[:n_dead], w[n_dead:n_dead + n_partial], w[n_dead + n_partial:n_dead + n_partial + n_inf],
                             w[n_dead + n_partial + n_inf:n_dead + n_partial + n_inf + 5])
    for k, ww in enumerate(np.concatenate([dead, pinw])):
        a, b = mo[ww], mo[ww + 1]
        comp = rng.integers(0, 3, b - a)
        pos[np.arange(a, b), comp] = np.nan
        if k % 3 == 1:
            vel[a:b] = np.nan
        if k % 3 == 2:
            pos[a:b, (comp + 1) % 3] = np.nan
    for ww in part:
        a, b = mo[ww], mo[ww + 1]
        pos[a:b - max(1, (b - a) // 2), 0] = np.nan
    for ww in inf:
        a, b = mo[ww], mo[ww + 1]
        pos[a:b, 1] = np.inf
    out = dict(spec, pos=pos, vel=vel)
    if pin:
        for ww in pinw:
            pinned[mo[ww]] = 1
        out["pinned"] = pinned
    return out


def _compare(spec, params, T, seed):
    import torch
    from oracle.oracle import Oracle
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    N = len(spec["mass_off"]) - 1
    A = max(1, int(np.max(spec["n_muscles"])))
    acts = np.random.default_rng(seed).uniform(-1, 1, (T, N, A)).astype(np.float32)
    env = BatchedPhysicsEnv(spec, **params)
    orc = Oracle(spec, params, n_threads=8)
    for t in range(T):
        obs, rew, done, info = env.step(acts[t])
        ref = orc.step(acts[t])
        torch.cuda.synchronize()
        _close(env.pos.cpu().numpy(), orc.pos)
        _close(env.vel.cpu().numpy(), orc.vel)
        _close(env.acc.cpu().numpy(), orc.acc)
        _close(env.muscle_x.cpu().numpy(), orc.mx)
        _close(obs.cpu().numpy(), ref["obs"])
        _close(rew.cpu().numpy(), ref["reward"])
        _close(info["centroid_position"].cpu().numpy(), ref["centroid"])
        _close(info["total_energy"].cpu().numpy(), ref["energy"])
        assert np.array_equal(done.cpu().numpy().astype(np.uint8), ref["done"])
        assert np.array_equal(env.contact.cpu().numpy(), orc.contact)
        assert np.array_equal(env.steps.cpu().numpy(), orc.steps)
    # the diverged walkers did diverge: the stand-in path ran (NaN in every component of every mass of some walker)
    p = env.pos.cpu().numpy()
    mo = np.asarray(spec["mass_off"])
    full = [bool(np.isnan(p[mo[w]:mo[w + 1]]).all()) for w in range(N)]
    assert sum(full) >= 20
    return env


def test_diverged_canonical_lean():
    from walker_gym_amd.synthetic import canonical_walkers
    spec = _diverge(canonical_walkers(512, seed=21), np.random.default_rng(1))
    _compare(spec, dict(in3d=1), 4, 5)


def test_diverged_balance_lean_ne1():
    from walker_gym_amd.walker import balance_spec
    spec = _diverge(balance_spec(1024), np.random.default_rng(2), n_dead=100, n_partial=60, n_inf=20)
    _compare(spec, dict(in3d=0), 4, 6)


def test_diverged_ragged_waves():
    from walker_gym_amd.synthetic import ragged_walkers
    spec = _diverge(ragged_walkers(600, seed=4, mmin=3, mmax=30, string_frac=0.1), np.random.default_rng(3))
    _compare(spec, dict(in3d=1, dampk=0.2), 4, 7)


def test_diverged_workgroup_kernel():
    """M = 25 walkers on the workgroup kernel (WG_LEAN=0: no stand-in path there) and pair forces on the lean kernel
    (stand-in path off): the diverged walkers step exactly."""
    import os
    from walker_gym_amd.synthetic import canonical_walkers
    spec = _diverge(canonical_walkers(200, seed=8, M=25, K=60, A=10), np.random.default_rng(4))
    old = os.environ.get("WG_LEAN")
    os.environ["WG_LEAN"] = "0"
    try:
        _compare(spec, dict(in3d=1), 3, 8)
    finally:
        if old is None:
            del os.environ["WG_LEAN"]
        else:
            os.environ["WG_LEAN"] = old
    spec = _diverge(canonical_walkers(256, seed=9), np.random.default_rng(5), pin=False)
    spec["charge"] = np.full(len(spec["m"]), 1e-6)
    _compare(spec, dict(in3d=1, pair_mode=3), 3, 9)


@pytest.mark.parametrize("workload", ["canonical", "balance"])
def test_diverged_resident_rollout_equals_steps(workload):
    """The resident rollout and per-step launches agree on diverged walkers: canonical (NE = 3: the resident kernel has
    no stand-in path) and Balance-v0 (NE = 1: both have it)."""
    import torch
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    from walker_gym_amd.walker import balance_spec
    if workload == "canonical":
        spec, kw = _diverge(canonical_walkers(1024, seed=31), np.random.default_rng(6), pin=False), dict(in3d=1)
    else:
        spec, kw = _diverge(balance_spec(2048), np.random.default_rng(7), n_dead=150, pin=False), dict(in3d=0)
    a, b = BatchedPhysicsEnv(spec, **kw), BatchedPhysicsEnv(spec, **kw)
    assert a.resident_ok()
    acts = (torch.rand((12, a.N, a.batch.A), device=a.device) * 2 - 1).contiguous()
    ro = a.rollout(acts, resident=True)
    rs = b.rollout(acts, resident=False)
    torch.cuda.synchronize()
    for x, y in zip(ro, rs):
        x, y = x.cpu().numpy(), y.cpu().numpy()
        if x.dtype == np.float32:
            _close(x, y)
        else:
            assert np.array_equal(x, y)
    for name in ("pos", "vel", "acc"):
        _close(getattr(a, name).cpu().numpy(), getattr(b, name).cpu().numpy())
