"""The C oracle against the drop-in-API fixtures (tests/golden/api, made by tests/golden/make_golden_api.py from
the reference's own PhysicsEnv / G1 Environment objects): seed -> reset noise -> steps, including every done
branch (max_steps, all-stopped after step 100, the 1,000-step rollout) and the G1 env's friction and step(t)."""
import glob
import os

import numpy as np
import pytest

from api_replay import api_creature, g1_creatures, g1_noise, physicsenv_noise
from conftest import GOLDEN

API = sorted(glob.glob(os.path.join(GOLDEN, "api", "api_*.npz")))


def _oracle_for(z):
    from oracle.oracle import Oracle
    from walker_gym_amd.walker import creatures_to_spec
    spec = creatures_to_spec([api_creature(str(z["env_id"]))])
    in3d = bool(int(z["kwargs_in3d"]))
    params = dict(in3d=int(in3d), dampk=float(z["kwargs_dampk"]), max_steps=int(z["max_steps"]))
    orc = Oracle(spec, params)
    P = int(spec["mass_off"][-1])
    n1, n2 = physicsenv_noise(P, float(z["kwargs_rand_sigma"]), in3d, int(z["np_seed_init"]), int(z["env_seed"]))
    orc.reset(n1)
    obs0 = orc.reset(n2)["obs"]
    return orc, obs0


@pytest.mark.parametrize("path", API, ids=[os.path.basename(p) for p in API])
def test_oracle_matches_physicsenv_fixture(path):
    z = np.load(path)
    orc, obs0 = _oracle_for(z)
    np.testing.assert_array_equal(obs0[0].astype(np.float64), z["out_obs0"])
    T = z["actions"].shape[0]
    every = 10 if z["out_pos"].shape[0] != T else 1          # api_rollout_1000 keeps every 10th state
    for t in range(T):
        ref = orc.step(z["actions"][t][None])
        assert ref["reward"][0] == z["out_reward"][t], t
        assert ref["done"][0] == z["out_done"][t], t
        assert ref["energy"][0] == z["out_energy"][t], t
        if (t + 1) % every == 0:
            s = (t + 1) // every - 1
            np.testing.assert_array_equal(ref["obs"][0].astype(np.float64), z["out_obs"][s])
            np.testing.assert_array_equal(ref["centroid"][0].astype(np.float64), z["out_centroid"][s])
            np.testing.assert_array_equal(orc.pos, z["out_pos"][s])
            np.testing.assert_array_equal(orc.vel, z["out_vel"][s])
            np.testing.assert_array_equal(orc.acc, z["out_acc"][s])
    # every done branch appears in some fixture
    if "maxsteps" in path:
        assert z["out_done"][39] == 1 and z["out_done"][:39].sum() == 0
    if "settle" in path:
        first = int(np.argmax(z["out_done"])) + 1
        assert first > 100 and np.abs(z["out_vel"][first - 1]).max() < 0.1
    if "1000" in path:
        assert z["out_done"][-1] == 1 and z["out_done"][:-1].sum() == 0


def test_oracle_matches_g1_environment_fixture():
    """gym/env.py Environment: random.gauss construction noise, G1 friction (friction_mode 1), step(t) with a
    varying t."""
    from oracle.oracle import Oracle
    from walker_gym_amd.walker import creatures_to_spec
    z = np.load(os.path.join(GOLDEN, "api", "g1_env.npz"))
    spec = creatures_to_spec(g1_creatures(z["g1_names"]))
    P = int(spec["mass_off"][-1])
    in3d = bool(int(z["in3d"]))
    orc = Oracle(spec, dict(in3d=int(in3d), dampk=float(z["dampk"]), friction_mode=1))
    orc.reset(g1_noise(P, float(z["randsigma"]), in3d, int(z["random_seed"])))
    np.testing.assert_array_equal(orc.vel, z["out_vel0"])
    for s, t in enumerate(z["ts"]):
        orc.params["dt"] = float(t)
        orc._mk_structs()
        orc.step(None, observe=False)
        np.testing.assert_array_equal(orc.pos, z["out_pos"][s])
        np.testing.assert_array_equal(orc.vel, z["out_vel"][s])
        np.testing.assert_array_equal(orc.acc, z["out_acc"][s])
