"""The reference-style per-object CPU loop (oracle/refstyle.py, bench.py's cpu_baseline) against the goldens
the reference itself produced: the same numbers, step by step."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.mark.parametrize("name,T", [("balance_3d", 100), ("canonical", 30), ("box_3d", 30), ("ragged", 20),
                                    ("pair_gravity_canonical", 20), ("perfdemo_chain_10", 40),
                                    ("pair_g2_gravity_canonical", 20)])
def test_refstyle_matches_golden(name, T):
    from oracle.oracle import spec_from_npz
    from oracle.refstyle import walkers
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    spec, params = spec_from_npz(z)
    ws = walkers(spec, params)
    for t in range(T):
        res = [wk.step(z["actions"][t, w] if z["actions"].shape[2] else []) for w, wk in enumerate(ws)]
        pos = np.array([p.pos for wk in ws for p in wk.phys])
        np.testing.assert_array_equal(pos, z["out_pos"][t])
        for w, (obs, rew, done, info) in enumerate(res):
            n = len(obs)
            np.testing.assert_array_equal(obs.astype(np.float32), z["out_obs"][t, w, :n])
            assert np.float32(rew) == z["out_reward"][t, w]
            assert int(done) == z["out_done"][t, w]


def test_refstyle_throughput_runs():
    from oracle.refstyle import throughput
    from walker_gym_amd.walker import balance_spec
    spec = balance_spec(4)
    acts = np.random.default_rng(0).uniform(-1, 1, (4, 4, 2)).astype(np.float32)
    r = throughput(spec, dict(in3d=0), acts, 0.3)
    assert r["value"] > 100 and r["procs"] == 1
