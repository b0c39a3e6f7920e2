"""The C oracle under AddressSanitizer + UBSan (host code): oracle/sanitize_check.c steps seeded ragged batches in
exactly-sized heap buffers through every mode (engine / G2 / G3 springs, strings, pinned masses, run1 / run2,
discrete actions, G1 friction, gravity / coulomb / bounce pairs), then observes and resets."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_under_asan_ubsan(tmp_path):
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize", f"OUT={tmp_path}"],
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    if r.returncode != 0 and ("cannot find -lasan" in r.stderr or "libasan" in r.stderr and "not found" in r.stderr):
        pytest.skip("no AddressSanitizer runtime in this toolchain")
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "sanitize ok" in r.stdout
