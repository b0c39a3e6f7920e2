"""ctypes binding of libwalker_hip.so (the C ABI in include/walker_hip.h).

The library is built in-tree (walker_gym_amd/libwalker_hip.so, see walker_gym_amd/build.py) so it
travels with the repo to the GPU box.  There is no fallback: if the library is missing or its ABI
version differs, every entry point raises — the product never silently runs on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libwalker_hip.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)
ABI_VERSION = 14

WG_EINVAL, WG_ERANGE, WG_EHIP = -1, -2, -3

_vp = C.c_void_p


class WgParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("g", "dampk", "ground", "groundk", "grounddamp", "friction", "dt",
                                           "pk", "vk", "ak", "mk")] + \
               [(n, C.c_int32) for n in ("in3d", "max_steps", "midform", "conmid", "spring_mode", "action_mode",
                                         "integrator", "pair_mode")] + \
               [(n, C.c_double) for n in ("pair_g", "pair_k", "pair_e", "bounce_k")] + \
               [("g3_gravity", C.c_double * 3)] + \
               [(n, C.c_double) for n in ("g3_damping", "g3_air", "g3_ground_level", "g3_restitution",
                                          "g3_friction")] + [("g3_ground", C.c_int32), ("friction_mode", C.c_int32)]


class WgBatch(C.Structure):
    _fields_ = [("N", C.c_int32), ("M", C.c_int32), ("K", C.c_int32), ("A", C.c_int32),
                ("ragged", C.c_int32),
                ("mass_off", _vp), ("edge_off", _vp), ("muscle_off", _vp),
                ("pos", _vp), ("vel", _vp), ("acc", _vp), ("mass", _vp),
                ("edges", _vp),
                ("inc", _vp), ("inc_off", _vp),
                ("muscle_x", _vp), ("muscle_bounds", _vp), ("muscle_stride", _vp),
                ("steps", _vp), ("contact", _vp), ("pinned", _vp),
                ("charge", _vp), ("radius", _vp), ("row", _vp), ("bounce_set", _vp)]


class WgOutputs(C.Structure):
    _fields_ = [("obs", _vp), ("obs_stride", C.c_int32), ("reward", _vp), ("done", _vp),
                ("centroid", _vp), ("energy", _vp), ("obs_step", C.c_int64), ("out_step", C.c_int64),
                ("obs_pad_clean", C.c_int32), ("steps", _vp), ("nonfinite", _vp), ("momentum", _vp)]


class WgRange(C.Structure):
    _fields_ = [("batch", C.POINTER(WgBatch)), ("outputs", C.POINTER(WgOutputs)), ("action_offset", C.c_int64),
                ("plan", _vp), ("plan_blocks", C.c_int32), ("stream", _vp)]


class WgLaunchInfo(C.Structure):
    _fields_ = [("threads", C.c_int32), ("walkers_per_block", C.c_int32), ("blocks", C.c_int32),
                ("lds_bytes", C.c_int32)]


EXPORTS = ("wg_abi_version", "wg_last_error", "wg_step", "wg_step_ranges", "wg_run_ranges", "wg_rollout", "wg_observe",
           "wg_step_simple", "wg_observe_simple", "wg_reset", "wg_reset_noise", "wg_plan_ragged", "wg_plan_waves",
           "wg_wave_edge_passes", "wg_plan_errors", "wg_launch_geometry", "wg_launch_floor", "wg_time_step")

_lib = None
_lock = threading.Lock()


class WalkerHipError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and type the library. Raises if it is missing or has the wrong ABI version."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("WALKER_HIP_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise WalkerHipError(
                f"{p} not found: build it with `python -m walker_gym_amd.build` (hipcc --offload-arch=gfx950); "
                "walker_gym_amd has no CPU fallback")
        L = C.CDLL(p)
        L.wg_abi_version.restype = C.c_int
        L.wg_last_error.restype = C.c_char_p
        L.wg_step.argtypes = [C.POINTER(WgBatch), C.POINTER(WgParams), _vp, C.c_int32, C.c_int32, C.c_int64,
                              C.POINTER(WgOutputs), C.c_int32, _vp, C.c_int32, _vp]
        L.wg_rollout.argtypes = L.wg_step.argtypes
        L.wg_step_ranges.argtypes = [C.POINTER(WgRange), C.c_int32, C.POINTER(WgParams), _vp, C.c_int32, C.c_int32,
                                     C.POINTER(_vp)]
        L.wg_run_ranges.argtypes = [C.POINTER(WgRange), C.c_int32, C.POINTER(WgParams), _vp, C.c_int32, C.c_int32,
                                    C.c_int64, C.c_int32, C.POINTER(_vp)]
        L.wg_observe.argtypes = [C.POINTER(WgBatch), C.POINTER(WgParams), C.POINTER(WgOutputs), _vp, C.c_int32, _vp]
        # SURVEY §8(b)'s declared signatures (ABI 13)
        L.wg_step_simple.argtypes = [C.POINTER(WgBatch), _vp, C.POINTER(WgParams), C.c_int32, _vp]
        L.wg_observe_simple.argtypes = [C.POINTER(WgBatch), C.POINTER(WgParams), _vp, _vp, _vp, _vp, _vp, _vp]
        L.wg_reset.argtypes = [C.POINTER(WgBatch), C.POINTER(WgParams), _vp, _vp, _vp]
        L.wg_reset_noise.argtypes = [C.POINTER(WgBatch), _vp, _vp]
        L.wg_plan_ragged.argtypes = [_vp, _vp, _vp, C.c_int32, _vp, C.c_int32]
        L.wg_plan_waves.argtypes = [_vp, _vp, _vp, C.c_int32, _vp, C.c_int32]
        L.wg_wave_edge_passes.argtypes = [C.c_int32, C.c_int32]
        L.wg_plan_errors.argtypes = [C.c_int32]
        L.wg_launch_geometry.argtypes = [C.POINTER(WgBatch), C.POINTER(WgLaunchInfo)]
        L.wg_launch_floor.argtypes = [C.c_int32, C.c_int32, C.c_int32, _vp, _vp, C.c_int32, _vp]
        L.wg_time_step.argtypes = L.wg_step.argtypes + [C.POINTER(C.c_float)]   # ABI 14, measurement aid
        for f in EXPORTS[2:]:
            getattr(L, f).restype = C.c_int
        v = L.wg_abi_version()
        if v != ABI_VERSION:
            raise WalkerHipError(f"{p}: ABI version {v}, expected {ABI_VERSION}")
        _lib = L
        return L


def check(rc: int, what: str) -> int:
    if rc < 0:
        msg = load().wg_last_error().decode(errors="replace")
        exc = ValueError if rc in (WG_EINVAL, WG_ERANGE) else WalkerHipError
        raise exc(f"{what}: {msg} (code {rc})")
    return rc
