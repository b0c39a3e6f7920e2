"""The C-ABI library loads, exports every symbol include/walker_hip.h declares, its ctypes structs match
the C layout, and its host-side validation / planning work without a GPU (no kernel is launched)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from walker_gym_amd import _lib, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "walker_hip.h")


@pytest.fixture(scope="module")
def lib():
    build.build()
    return _lib.load()


def declared_functions():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(wg_\w+)\s*\(", src, re.M)))


def test_every_declared_symbol_is_exported(lib):
    names = declared_functions()
    assert {"wg_step", "wg_observe", "wg_reset", "wg_abi_version", "wg_last_error"} <= set(names)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (wg_\w+)", out))
    assert set(names) <= exported, set(names) - exported
    assert set(_lib.EXPORTS) <= exported


def test_abi_version(lib):
    assert lib.wg_abi_version() == _lib.ABI_VERSION
    assert f"#define WG_ABI_VERSION {_lib.ABI_VERSION}" in open(HDR).read()


def test_struct_layout_matches_header(tmp_path):
    """Compile a C probe against the header and compare sizeof/offsetof with the ctypes mirrors."""
    probe = tmp_path / "probe.c"
    probe.write_text("""
#include <stdio.h>
#include <stddef.h>
#include "walker_hip.h"
#define F(T, m) printf(#T "." #m " %zu\\n", offsetof(T, m));
int main(void) {
  printf("wg_params %zu\\nwg_batch %zu\\nwg_outputs %zu\\nwg_edge %zu\\nwg_launch_info %zu\\n",
         sizeof(wg_params), sizeof(wg_batch), sizeof(wg_outputs), sizeof(wg_edge), sizeof(wg_launch_info));
  F(wg_batch, pos) F(wg_batch, edges) F(wg_batch, inc_off) F(wg_batch, muscle_bounds) F(wg_batch, contact)
  F(wg_outputs, obs_step) F(wg_outputs, out_step) F(wg_params, in3d) F(wg_params, action_mode) F(wg_params, pair_g)
  F(wg_params, bounce_k) F(wg_batch, charge) F(wg_batch, radius) F(wg_batch, row) F(wg_batch, bounce_set)
  printf("wg_range %zu\\n", sizeof(wg_range));
  F(wg_range, outputs) F(wg_range, action_offset) F(wg_range, plan) F(wg_range, plan_blocks) F(wg_range, stream)
  return 0;
}
""")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(probe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True)
               .stdout.strip().splitlines())
    assert int(got["wg_params"]) == C.sizeof(_lib.WgParams)
    assert int(got["wg_batch"]) == C.sizeof(_lib.WgBatch)
    assert int(got["wg_outputs"]) == C.sizeof(_lib.WgOutputs)
    assert int(got["wg_launch_info"]) == C.sizeof(_lib.WgLaunchInfo)
    assert int(got["wg_edge"]) == 16
    assert int(got["wg_range"]) == C.sizeof(_lib.WgRange)
    for key, cls in (("wg_batch", _lib.WgBatch), ("wg_outputs", _lib.WgOutputs), ("wg_params", _lib.WgParams),
                     ("wg_range", _lib.WgRange)):
        for full, off in got.items():
            if full.startswith(key + "."):
                assert getattr(cls, full.split(".", 1)[1]).offset == int(off), full


def test_errors_without_gpu(lib):
    p = _lib.WgParams()
    assert lib.wg_step(None, C.byref(p), None, 0, 0, 0, None, 1, None, 0, None) == _lib.WG_EINVAL
    assert b"null batch" in lib.wg_last_error()
    b = _lib.WgBatch(N=4, M=0, K=1, A=0)
    assert lib.wg_step(C.byref(b), C.byref(p), None, 0, 0, 0, None, 1, None, 0, None) == _lib.WG_EINVAL
    b = _lib.WgBatch(N=4, M=2000, K=1, A=0)
    assert lib.wg_step(C.byref(b), C.byref(p), None, 0, 0, 0, None, 1, None, 0, None) == _lib.WG_ERANGE
    with pytest.raises(ValueError):
        _lib.check(-1, "probe")
    assert lib.wg_reset_noise(None, None, None) == _lib.WG_EINVAL
    # SURVEY §8(b)'s declared signatures (ABI 13): the same checks, and ragged batches refused (no plan argument)
    assert lib.wg_step_simple(None, None, C.byref(p), 1, None) == _lib.WG_EINVAL
    assert b"null batch" in lib.wg_last_error()
    assert lib.wg_observe_simple(C.byref(_lib.WgBatch(N=4, M=8, K=4, A=0)), None, None, None, None, None, None,
                                 None) == _lib.WG_EINVAL
    rb = _lib.WgBatch(N=4, M=8, K=4, A=0, ragged=2)
    assert lib.wg_step_simple(C.byref(rb), None, C.byref(p), 1, None) == _lib.WG_EINVAL
    assert b"uniform batches only" in lib.wg_last_error()
    assert lib.wg_observe_simple(C.byref(rb), C.byref(p), None, None, None, None, None, None) == _lib.WG_EINVAL
    # the measurement aid (ABI 14): an output pointer and n_steps >= 1 required, the batch checked as wg_step checks it
    ms = C.c_float(-1.0)
    assert lib.wg_time_step(None, C.byref(p), None, 0, 0, 0, None, 1, None, 0, None, C.byref(ms)) == _lib.WG_EINVAL
    assert b"ms_per_launch" in lib.wg_last_error() or b"null batch" in lib.wg_last_error()
    ub = _lib.WgBatch(N=4, M=8, K=4, A=0)
    assert lib.wg_time_step(C.byref(ub), C.byref(p), None, 0, 0, 0, None, 0, None, 0, None, C.byref(ms)) == _lib.WG_EINVAL
    assert lib.wg_time_step(C.byref(ub), C.byref(p), None, 0, 0, 0, None, 1, None, 0, None, None) == _lib.WG_EINVAL
    assert b"ms_per_launch" in lib.wg_last_error()
    assert lib.wg_time_step(C.byref(ub), C.byref(p), None, 0, 0, 0, None, 1, None, 0, None, C.byref(ms)) == _lib.WG_EINVAL
    assert b"missing state pointer" in lib.wg_last_error() and ms.value == -1.0
    # pair passes need the engine.py spring (spring_mode 0): refused before any launch
    b = _lib.WgBatch(N=4, M=8, K=4, A=0, ragged=1)
    for f in ("pos", "vel", "acc", "mass", "edges", "inc", "inc_off", "muscle_x", "steps", "mass_off", "edge_off",
              "muscle_off"):
        setattr(b, f, 16)
    p = _lib.WgParams(pair_mode=1, pair_g=9.8, spring_mode=1)
    plan = np.zeros(2, np.int32)
    assert lib.wg_step(C.byref(b), C.byref(p), None, 0, 0, 0, None, 1, plan.ctypes.data_as(C.c_void_p), 1, None) == _lib.WG_EINVAL
    assert b"pair_mode" in lib.wg_last_error()
    # ragged kinds: 0, 1 (workgroup plan), 2 (wave plan, M <= 64 only); a walker permutation only for ragged batches
    p = _lib.WgParams()
    for kind, M in ((3, 8), (2, 65)):
        b.ragged, b.M = kind, M
        assert lib.wg_step(C.byref(b), C.byref(p), None, 0, 0, 0, None, 1, plan.ctypes.data_as(C.c_void_p), 1,
                           None) == _lib.WG_EINVAL
    b.ragged, b.M, b.row = 0, 8, 16
    assert lib.wg_step(C.byref(b), C.byref(p), None, 0, 0, 0, None, 1, None, 0, None) == _lib.WG_EINVAL
    assert b"row" in lib.wg_last_error()
    b.row = None
    # unknown pair bits, and bounce without the radius array, are refused before any launch
    b.ragged = 0
    for pm in (32, 64 | 1, 4):
        p = _lib.WgParams(pair_mode=pm, bounce_k=100.0)
        assert lib.wg_step(C.byref(b), C.byref(p), None, 0, 0, 0, None, 1, None, 0, None) == _lib.WG_EINVAL
        assert b"pair_mode" in lib.wg_last_error()


def test_plan_ragged_host(lib):
    rng = np.random.default_rng(0)
    N = 500
    Ms = rng.integers(2, 40, N); Ks = rng.integers(1, 80, N); As = Ks // 5
    mo = np.concatenate([[0], np.cumsum(Ms)]).astype(np.int32)
    eo = np.concatenate([[0], np.cumsum(Ks)]).astype(np.int32)
    uo = np.concatenate([[0], np.cumsum(As)]).astype(np.int32)
    plan = np.zeros(N + 1, np.int32)
    nb = lib.wg_plan_ragged(mo.ctypes.data_as(C.c_void_p), eo.ctypes.data_as(C.c_void_p),
                            uo.ctypes.data_as(C.c_void_p), N, plan.ctypes.data_as(C.c_void_p), N + 1)
    assert nb > 0 and plan[0] == 0 and plan[nb] == N
    for k in range(nb):
        a, b = plan[k], plan[k + 1]
        assert b > a
        if b - a > 1:   # multi-walker blocks respect the caps
            assert mo[b] - mo[a] <= 256 and eo[b] - eo[a] <= 512 and b - a <= 64


def test_launch_geometry_canonical(lib):
    b = _lib.WgBatch(N=65536, M=16, K=40, A=8, ragged=0)
    for f in ("pos", "vel", "acc", "mass", "edges", "inc", "inc_off", "muscle_x", "steps"):
        setattr(b, f, 16)   # non-null placeholders; nothing is dereferenced on the host
    info = _lib.WgLaunchInfo()
    assert lib.wg_launch_geometry(C.byref(b), C.byref(info)) == 0
    assert info.threads == 256 and info.walkers_per_block == 16 and info.blocks == 4096
    assert info.lds_bytes <= 32768   # five workgroups per CU (160 KiB LDS)


def test_launch_geometry_wave_tiles(lib):
    """ragged = 2 (sorted wave tiles): the wave kernel's geometry, 4 waves per workgroup and its LDS slices; the tile
    count comes from the plan, so blocks and walkers per block are -1."""
    b = _lib.WgBatch(N=1000, M=32, K=64, A=12, ragged=2)
    for f in ("pos", "vel", "acc", "mass", "edges", "inc", "inc_off", "muscle_x", "steps", "mass_off", "edge_off",
              "muscle_off"):
        setattr(b, f, 16)
    info = _lib.WgLaunchInfo()
    assert lib.wg_launch_geometry(C.byref(b), C.byref(info)) == 0
    assert info.threads == 256 and info.walkers_per_block == -1 and info.blocks == -1
    assert 4 * 5 * 1024 <= info.lds_bytes <= 4 * 7 * 1024   # ~5.9 KB per wave at 2 spring passes


def test_launch_geometry_wide_workgroups(lib, monkeypatch):
    """M > 64: the workgroup size in 256..512 threads that leaves the fewest idle lanes (walker_hip.hip
    uniform_geo), halved back while the grid has fewer than 512 workgroups; WG_WIDE=0 keeps 256."""
    def geo(N, M, K):
        b = _lib.WgBatch(N=N, M=M, K=K, A=0, ragged=0)
        for f in ("pos", "vel", "acc", "mass", "edges", "inc", "inc_off", "muscle_x", "steps"):
            setattr(b, f, 16)
        info = _lib.WgLaunchInfo()
        assert lib.wg_launch_geometry(C.byref(b), C.byref(info)) == 0
        return info.threads, info.walkers_per_block
    assert geo(4096, 100, 99) == (512, 5)      # the performance_demo chain: 500 of 512 lanes busy
    assert geo(4096, 200, 199) == (448, 2)
    assert geo(4096, 128, 127) == (256, 2)
    assert geo(40, 100, 99) == (128, 1)        # small batch: more, smaller workgroups
    monkeypatch.setenv("WG_WIDE", "0")
    assert geo(4096, 100, 99) == (256, 2)


def test_wave_edge_passes(lib):
    """Spring passes of a wave tile (walker_hip.hip wave_passes): enough for the longest walker and for 64 masses of
    the densest one, rounded to an instantiated count; 0 = the batch cannot use the wave kernel."""
    for (M, K), ne in {(32, 64): 2, (16, 40): 3, (4, 5): 2, (8, 4): 1, (64, 300): 8, (64, 512): 8,
                       (65, 10): 0, (4, 600): 0, (2, 20): 0}.items():
        assert lib.wg_wave_edge_passes(M, K) == ne, (M, K)


def test_plan_waves_host(lib):
    rng = np.random.default_rng(1)
    N = 3000
    Ms = rng.integers(1, 33, N); Ks = np.minimum(rng.integers(0, 2 * Ms + 1), 64); As = Ks // 5
    mo = np.concatenate([[0], np.cumsum(Ms)]).astype(np.int32)
    eo = np.concatenate([[0], np.cumsum(Ks)]).astype(np.int32)
    uo = np.concatenate([[0], np.cumsum(As)]).astype(np.int32)
    ne = lib.wg_wave_edge_passes(int(Ms.max()), int(Ks.max()))
    assert ne > 0
    plan = np.zeros(N + 1, np.int32)
    args = (mo.ctypes.data_as(C.c_void_p), eo.ctypes.data_as(C.c_void_p), uo.ctypes.data_as(C.c_void_p), N)
    nt = lib.wg_plan_waves(*args, plan.ctypes.data_as(C.c_void_p), N + 1)
    assert nt > 0 and plan[0] == 0 and plan[nt] == N
    a, b = plan[:nt], plan[1:nt + 1]
    assert np.all(b > a) and np.all(b - a <= 32)                       # RW_MAXW walkers per tile
    assert np.all(mo[b] - mo[a] <= 64) and np.all(uo[b] - uo[a] <= 64) and np.all(eo[b] - eo[a] <= 64 * ne)
    # greedy and maximal: the next walker would not have fitted any tile but the last
    nxt = b[:-1]
    full = ((mo[nxt + 1] - mo[a[:-1]] > 64) | (eo[nxt + 1] - eo[a[:-1]] > 64 * ne) | (uo[nxt + 1] - uo[a[:-1]] > 64)
            | (nxt + 1 - a[:-1] > 32))
    assert np.all(full)
    small = np.zeros(2, np.int32)
    assert lib.wg_plan_waves(*args, small.ctypes.data_as(C.c_void_p), 1) == _lib.WG_ERANGE
    big = np.array([0, 65], np.int32)
    assert lib.wg_plan_waves(big.ctypes.data_as(C.c_void_p), np.array([0, 4], np.int32).ctypes.data_as(C.c_void_p),
                             np.array([0, 0], np.int32).ctypes.data_as(C.c_void_p), 1,
                             small.ctypes.data_as(C.c_void_p), 1) == _lib.WG_EINVAL


def test_launch_geometry_small_batch_halves_tiles(lib):
    """A uniform batch with fewer than 512 full wave tiles gets fewer walkers per wave (two tiles per CU), and a batch
    of at most 1,024 tiles one wave per workgroup (the tiles spread over every CU)."""
    b = _lib.WgBatch(N=4096, M=4, K=5, A=2, ragged=0)
    for f in ("pos", "vel", "acc", "mass", "edges", "inc", "inc_off", "muscle_x", "steps"):
        setattr(b, f, 16)
    info = _lib.WgLaunchInfo()
    assert lib.wg_launch_geometry(C.byref(b), C.byref(info)) == 0
    assert info.walkers_per_block == 8 and info.blocks == 512 and info.threads == 64   # 8 Balance walkers per wave


def test_step_ranges_argument_errors(lib):
    """wg_step_ranges (ABI 8) refuses bad range lists before touching a stream: no ranges, n < 1, n > 1 without
    events, and a range whose batch is invalid (the per-range wg_step checks)."""
    p = _lib.WgParams()
    assert lib.wg_step_ranges(None, 1, C.byref(p), None, 0, 0, None) == _lib.WG_EINVAL
    rng = (_lib.WgRange * 2)()
    assert lib.wg_step_ranges(rng, 0, C.byref(p), None, 0, 0, None) == _lib.WG_EINVAL
    assert lib.wg_step_ranges(rng, 2, C.byref(p), None, 0, 0, None) == _lib.WG_EINVAL
    assert b"events" in lib.wg_last_error()
    bad = _lib.WgBatch(N=4, M=0, K=1, A=0)
    rng[0].batch = C.pointer(bad)
    assert lib.wg_step_ranges(rng, 1, C.byref(p), None, 0, 0, None) == _lib.WG_EINVAL


def test_build_switches_are_diagnostic_only():
    """every A/B build switch whose non-default arm lost was deleted with its arm; what is left is the
    diagnostic WG_ABLATE (phase ablation, timing builds whose results are not exact) and the #ifdef WG_STAMPS phase
    timeline.  Both still compile for gfx950 (device code only, together)."""
    import re
    import subprocess
    src = os.path.join(ROOT, "walker_gym_amd", "csrc", "walker_hip.hip")
    text = open(src).read()
    switches = re.findall(r"#ifndef (WG_\w+)", text)
    assert switches == ["WG_ABLATE"], switches
    assert set(re.findall(r"#ifdef (WG_\w+)", text)) == {"WG_STAMPS"}
    assert "results are NOT exact" in text            # the header says what such builds are
    from walker_gym_amd import build as wb
    cmd = [wb.hipcc(), f"--offload-arch={wb.ARCH}", "-O1", "-std=c++17", "-ffp-contract=off",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero", "--cuda-device-only", "-c",
           "-o", os.devnull, "-DWG_ABLATE=4095", "-DWG_STAMPS", "-I", os.path.join(ROOT, "include"), src]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
