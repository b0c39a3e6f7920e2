#!/usr/bin/env python3
"""Per-workgroup phase timeline of the generic step kernel (diagnostic build with -DWG_STAMPS).
build: python scripts/stamps.py build     run (GPU): python scripts/stamps.py run"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "build_ablate", "lib_stamps.so")
NAMES = ["start", "loads+act", "edge", "mass", "reduce", "obs-tile", "end"]


def build(extra=()):
    from walker_gym_amd import build as wb
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    cmd = wb.command(LIB)
    cmd = cmd[:-1] + ["-DWG_STAMPS", *extra] + cmd[-1:]
    subprocess.run(cmd, check=True)


def run(n=int(os.environ.get("WG_N", "65536"))):
    os.environ["WALKER_HIP_LIB"] = LIB
    import torch
    from walker_gym_amd import _lib
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    L = _lib.load()
    L.wg_debug_stamps.argtypes = [C.c_void_p, C.c_int]
    env = BatchedPhysicsEnv(canonical_walkers(n, seed=0), in3d=1)
    acts = (torch.rand((6, n, 8), device="cuda") * 2 - 1).contiguous()
    env.run(acts[:5].contiguous(), 5)
    torch.cuda.synchronize()
    env.run(acts[5:].contiguous(), 1)
    torch.cuda.synchronize()
    nb = env.launch_geometry()["blocks"]
    st = np.zeros((nb, 16), np.uint64)
    assert L.wg_debug_stamps(st.ctypes.data_as(C.c_void_p), nb) == 0
    t = (st[:, :7].astype(np.int64) - int(st[:, 0].min())) / 100.0   # us (100 MHz)
    print(f"blocks {nb}; kernel span {t[:, 6].max():.1f} us; block start spread {t[:, 0].max():.1f} us")
    d = np.diff(t, axis=1)
    for k in range(6):
        print(f"  {NAMES[k]:>10s} -> {NAMES[k+1]:<10s} mean {d[:, k].mean():6.2f}  p50 {np.median(d[:, k]):6.2f}"
              f"  p90 {np.percentile(d[:, k], 90):6.2f} us")
    tt = (st.astype(np.int64) - int(st[:, 0].min())) / 100.0
    for a, b_, nm in ((2, 10, "edge-end -> mass start (1/m)"), (10, 7, "incidence loop"), (7, 8, "env+run1"),
                      (8, 9, "stores+norm+seq/pw sums"), (9, 3, "ballots+outputs+barrier")):
        dd = tt[:, b_] - tt[:, a]
        print(f"  {nm:>32s} mean {dd.mean():6.2f} p50 {np.median(dd):6.2f} us")
    life = t[:, 6] - t[:, 0]
    print(f"  block lifetime mean {life.mean():.2f} p50 {np.median(life):.2f} p90 {np.percentile(life, 90):.2f}")
    # concurrency profile
    edges = np.linspace(0, t[:, 6].max(), 21)
    conc = [int(((t[:, 0] <= x) & (t[:, 6] > x)).sum()) for x in edges[:-1]]
    print("  resident blocks over time:", conc)


def run_lean(n=int(os.environ.get("WG_N", "65536"))):
    """Lean kernel (default path): wave 0 of each workgroup stamps its tile's phases."""
    os.environ["WALKER_HIP_LIB"] = LIB
    import torch
    from walker_gym_amd import _lib
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.synthetic import canonical_walkers
    L = _lib.load()
    L.wg_debug_stamps.argtypes = [C.c_void_p, C.c_int]
    env = BatchedPhysicsEnv(canonical_walkers(n, seed=0), in3d=1)
    acts = (torch.rand((30, n, 8), device="cuda") * 2 - 1).contiguous()
    env.run(acts[:29].contiguous(), 29)
    torch.cuda.synchronize()
    env.run(acts[29:].contiguous(), 1)
    torch.cuda.synchronize()
    nb = env.launch_geometry()["blocks"]
    st = np.zeros((nb, 16), np.uint64)
    assert L.wg_debug_stamps(st.ctypes.data_as(C.c_void_p), nb) == 0
    tt = (st.astype(np.int64) - int(st[:, 0].min())) / 100.0   # us (100 MHz)
    seq = [(0, "compute start (loads issued)"), (1, "act done: loads landed"), (2, "springs"), (10, "mass loop start"),
           (7, "mass loop end"), (8, "env forces + run1"), (9, "reductions"), (3, "state/output stores"),
           (5, "obs tile"), (6, "obs stores")]
    print(f"blocks {nb}; span {tt[:, 6].max():.1f} us; start spread {tt[:, 0].max():.1f} us")
    for (a, na), (b_, nb_) in zip(seq[:-1], seq[1:]):
        d = tt[:, b_] - tt[:, a]
        print(f"  {na:>30s} -> {nb_:<30s} mean {d.mean():6.2f}  p50 {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f} us")
    life = tt[:, 6] - tt[:, 0]
    print(f"  wave-0 lifetime mean {life.mean():.2f} p50 {np.median(life):.2f} p90 {np.percentile(life, 90):.2f} us")
    edges = np.linspace(0, tt[:, 6].max(), 21)
    print("  resident (stamped) tiles over time:", [int(((tt[:, 0] <= x) & (tt[:, 6] > x)).sum()) for x in edges[:-1]])


if __name__ == "__main__":
    {"build": build, "run": run, "lean": run_lean}[sys.argv[1]]()
