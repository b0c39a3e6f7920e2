"""bench.py's rank launcher, on the CPU: `--gpus N` outside a torch.distributed world starts N
rank processes itself (torch.distributed.run; --dry-run stops before any GPU call and makes every rank report
itself over a gloo barrier), and a world whose size differs from --gpus is refused with exit status 2."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                               "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_2_launches_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"dry_run"')]
    assert sorted(l["rank"] for l in lines) == [0, 1], r.stdout[-2000:]
    assert all(l["world"] == 2 and l["gpus"] == 2 for l in lines)


def test_single_gpu_needs_no_launcher():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"dry_run"')]
    assert len(lines) == 1 and lines[0]["world"] == 1


def test_world_size_mismatch_exits_2():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=_env(WORLD_SIZE="3", RANK="0"))
    assert r.returncode == 2
    assert "world has 3 ranks" in r.stderr
