"""state.pkl is read by walking opcodes — nothing in the file is executed."""
import io
import os
import pickle

import numpy as np
import pytest

from walker_gym_amd.snapshot import SnapshotError, read_snapshot, read_snapshot_bytes, write_snapshot

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_reads_reference_state_pkl():
    pts, rp = read_snapshot(os.path.join(GOLDEN, "state.pkl"))
    assert len(pts) == 2 and rp == {}
    assert [p.m for p in pts] == [1.0, 1.0]
    assert np.array_equal(pts[0].pos, [0, 0, 0]) and np.array_equal(pts[1].pos, [0, 0, 1])
    assert np.array_equal(pts[0].v, [1, 0, 0]) and pts[0].pos.dtype == np.float32


def test_write_read_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    m = rng.uniform(1, 5, 7)
    pos, v = rng.standard_normal((7, 3)).astype(np.float32), rng.standard_normal((7, 3)).astype(np.float32)
    path = str(tmp_path / "s.pkl")
    write_snapshot(path, m, pos, v)
    pts, _ = read_snapshot(path)
    assert np.allclose([p.m for p in pts], m)
    assert np.array_equal(np.stack([p.pos for p in pts]), pos)
    assert np.array_equal(np.stack([p.v for p in pts]), v)


def test_malicious_pickle_is_not_executed(tmp_path):
    marker = tmp_path / "pwned"

    class Evil:
        def __reduce__(self):
            return (os.system, (f"touch {marker}",))

    data = pickle.dumps({"points": [Evil()], "r_points": {}}, protocol=4)
    with pytest.raises(SnapshotError):
        read_snapshot_bytes(data)
    assert not marker.exists()
    with pytest.raises(SnapshotError):
        read_snapshot_bytes(pickle.dumps([1, 2, 3], protocol=4))
    assert io is not None
