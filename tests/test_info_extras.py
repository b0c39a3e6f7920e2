"""The opt-in info outputs (ABI 10) on the CPU side: the momentum restatement (oracle.momentum, gym/engine.py:160-166)
and the non-finite flag (oracle.nonfinite) against the reference's own Point.momentum() values and states recorded
in tests/golden/info_extras.npz (make_golden.py scenario info_extras: two Box-v0 walkers, one of which goes
non-finite at step 27, beside two Balance-v0 walkers), bit for bit."""
import os

import numpy as np

from oracle.oracle import momentum, nonfinite

Z = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "info_extras.npz")


def _bits_or_nan(a, b):
    a, b = np.ascontiguousarray(a, np.float32), np.ascontiguousarray(b, np.float32)
    return ((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))).all()


def test_momentum_restatement_matches_reference():
    z = np.load(Z)
    for t in range(z["out_momentum"].shape[0]):
        assert _bits_or_nan(momentum(z["out_vel"][t], z["in_m"], z["in_mass_off"]), z["out_momentum"][t]), t


def test_nonfinite_flag_pattern():
    z = np.load(Z)
    flags = np.array([nonfinite(z["out_pos"][t], z["out_vel"][t], z["out_acc"][t], z["in_mass_off"])
                      for t in range(z["out_pos"].shape[0])])
    first = int(np.argmax(flags[:, 1]))
    assert flags[first:, 1].all() and not flags[:first, 1].any()     # walker 1 diverges and stays non-finite
    assert not flags[:, [0, 2, 3]].any()                              # the others stay finite
    assert not np.isfinite(z["out_momentum"][first:, 1]).all()
    # the reference's done does not test finiteness (gym/optimized_env.py:207-230): it stays 0 for the NaN walker
    assert not z["out_done"][first:, 1].any()
