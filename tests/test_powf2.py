"""numpy's float32 `x ** 2` is libm powf, not x*x (e.g. powf(673.88745f, 2) = 454124.3125f, x*x = 454124.28125f).
The kernel restates glibc's powf at y = 2 (walker_gym_amd/csrc/powf2.h) for the energy term
(gym/optimized_env.py:242) and Point.gravity_vec's distance ** 2 (gym/optimized_engine.py:189).  This checks the
restatement, compiled for the host from the same header, against the image's libm powf: every 5th non-negative
finite float and its negation here (the full sweep over all 4,278,190,080 inputs is profiles/r03_powf2_exhaustive.json,
`scripts/check_powf2 1`), and that the fast path's claim (RN(x*x) when x^2 is 2^-32 away from a rounding boundary)
never disagrees with libm."""
import ctypes
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_libm_powf_is_not_x_times_x():
    libm = ctypes.CDLL("libm.so.6")
    libm.powf.restype, libm.powf.argtypes = ctypes.c_float, [ctypes.c_float, ctypes.c_float]
    x = np.float32(673.88745)
    assert np.float32(libm.powf(float(x), 2.0)) == x ** 2 != x * x


def test_powf2_restatement_matches_libm(tmp_path):
    exe = str(tmp_path / "check_powf2")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-fno-builtin", "-I",
                    os.path.join(ROOT, "walker_gym_amd", "csrc"), "-o", exe,
                    os.path.join(ROOT, "scripts", "check_powf2.c"), "-lm"], check=True)
    r = subprocess.run([exe, "5"], capture_output=True, text=True, timeout=300)
    res = json.loads(r.stdout)
    assert r.returncode == 0 and res["mismatch"] == 0 and res["fast_mismatch"] == 0, res
    assert res["inputs"] > 8e8 and res["slow_path"] < 0.004 * res["inputs"], res
