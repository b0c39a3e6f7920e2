"""The committed fixtures regenerate from HEAD: one cheap scenario of each generator script is
rerun against /root/reference into a temporary directory and every array of the result must equal the committed
file's — same keys, dtypes, shapes and bytes.  (The .npz containers themselves differ in their zip timestamps, so
the comparison is of the arrays, not of the archive bytes.)  Each fixture draws from its own name-seeded generator
(make_golden.scenario_rng), so this holds for every fixture, not only for these.  Skipped where the reference is
absent (the GPU box)."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF = "/root/reference"

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "gym")), reason="reference not present")


def _same_arrays(a_path, b_path):
    a, b = np.load(a_path), np.load(b_path)
    assert sorted(a.files) == sorted(b.files)
    for k in a.files:
        x, y = a[k], b[k]
        assert x.dtype == y.dtype and x.shape == y.shape, k
        assert x.tobytes() == y.tobytes(), k


@pytest.mark.parametrize("script,fixtures", [
    ("make_golden.py", ["state_pkl"]),
    ("make_golden.py", ["balance_2d", "balance_3d"]),
    ("make_golden_api.py", ["api_balance_2d"]),
])
def test_fixture_regenerates_identically(tmp_path, script, fixtures):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, os.path.join(GOLDEN, script), "--ref", REF, "--out", str(tmp_path),
                        "--only", *fixtures], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    sub = "api" if script == "make_golden_api.py" else ""
    for name in fixtures:
        _same_arrays(os.path.join(tmp_path, name + ".npz"), os.path.join(GOLDEN, sub, name + ".npz"))
