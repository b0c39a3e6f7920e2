"""ctypes front-end of the CPU oracle (liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / the reported CPU baseline.  The product (walker_gym_amd) never imports it.
The arithmetic lives in walker_oracle.c, which cites the reference file:line it restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_i32p = C.POINTER(C.c_int32)
_f32p = C.POINTER(C.c_float)
_u8p = C.POINTER(C.c_uint8)
_f64p = C.POINTER(C.c_double)


class OrcParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("g", "dampk", "ground", "groundk", "grounddamp", "friction",
                                           "dt", "pk", "vk", "ak", "mk")] + \
               [(n, C.c_int32) for n in ("in3d", "max_steps", "midform", "conmid", "spring_mode",
                                         "action_mode", "integrator", "pair_mode")] + \
               [(n, C.c_double) for n in ("pair_g", "pair_k", "pair_e", "bounce_k")] + \
               [("g3_gravity", C.c_double * 3)] + \
               [(n, C.c_double) for n in ("g3_damping", "g3_air", "g3_ground_level", "g3_restitution",
                                          "g3_friction")] + [("g3_ground", C.c_int32), ("friction_mode", C.c_int32)]


class OrcBatch(C.Structure):
    _fields_ = [("N", C.c_int32), ("mass_off", _i32p), ("edge_off", _i32p), ("muscle_off", _i32p),
                ("pos", _f32p), ("vel", _f32p), ("acc", _f32p), ("m", _f32p),
                ("ei", _i32p), ("ej", _i32p), ("rest", _f32p), ("k", _f32p), ("c", _f32p),
                ("flags", _u8p), ("mx", _f32p), ("minl", _f32p), ("maxl", _f32p), ("stride", _f32p),
                ("steps", _i32p), ("contact", _u8p), ("pinned", _u8p),
                ("charge", _f64p), ("radius", _f64p), ("bounce_set", _u8p)]


class OrcOut(C.Structure):
    _fields_ = [("obs", _f32p), ("obs_stride", C.c_int32), ("reward", _f32p), ("done", _u8p),
                ("centroid", _f32p), ("energy", _f32p)]


_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "walker_oracle.c")):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        L.orc_step.argtypes = [C.POINTER(OrcBatch), C.POINTER(OrcParams), _f32p, C.c_int32, C.c_int32,
                               C.POINTER(OrcOut), C.c_int32]
        L.orc_observe.argtypes = [C.POINTER(OrcBatch), C.POINTER(OrcParams), C.POINTER(OrcOut), C.c_int32]
        L.orc_reset.argtypes = [C.POINTER(OrcBatch), C.POINTER(OrcParams), _f32p, C.c_int32]
        L.orc_np_norm3.argtypes = [_f32p]; L.orc_np_norm3.restype = C.c_float
        L.orc_np_pairwise_sum.argtypes = [_f32p, C.c_int64, C.c_int64]
        L.orc_np_pairwise_sum.restype = C.c_float
        _lib = L
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


DEFAULT_PARAMS = dict(g=100.0, dampk=0.0, ground=0.0, groundk=1000.0, grounddamp=100.0, friction=100.0,
                      dt=0.01, in3d=1, max_steps=1000, pk=1.0, vk=1.0, ak=1.0, mk=1.0, midform=1,
                      conmid=0, spring_mode=0, action_mode=0, integrator=1, pair_mode=0, pair_g=9.8,
                      pair_k=8.99e9, pair_e=16e-20, bounce_k=100.0,
                      g3_gravity=(0.0, -9.8, 0.0), g3_damping=0.99, g3_air=0.01, g3_ground_level=-50.0,
                      g3_restitution=0.8, g3_friction=0.5, g3_ground=1, friction_mode=0)


class Oracle:
    """Holds one batch (flat CSR arrays, numpy) and steps it with the C restatement."""

    def __init__(self, spec: dict, params: dict | None = None, n_threads: int = 1):
        P = dict(DEFAULT_PARAMS)
        if params:
            P.update({k: v for k, v in params.items() if k in P})
        self.params = P
        s = {k: np.asarray(v) for k, v in spec.items()}
        self.mass_off = np.ascontiguousarray(s["mass_off"], np.int32)
        self.edge_off = np.ascontiguousarray(s["edge_off"], np.int32)
        self.n_muscles = np.ascontiguousarray(s["n_muscles"], np.int32)
        self.muscle_off = np.concatenate([[0], np.cumsum(self.n_muscles)]).astype(np.int32)
        self.N = len(self.mass_off) - 1
        self.pos = np.ascontiguousarray(s["pos"], np.float32).reshape(-1, 3).copy()
        self.vel = np.ascontiguousarray(s["vel"], np.float32).reshape(-1, 3).copy()
        acc = s.get("acc")
        self.acc = (np.zeros_like(self.pos) if acc is None
                    else np.ascontiguousarray(acc, np.float32).reshape(-1, 3).copy())
        self.m = np.ascontiguousarray(s["m"], np.float32)
        self.ei = np.ascontiguousarray(s["ei"], np.int32)
        self.ej = np.ascontiguousarray(s["ej"], np.int32)
        self.rest = np.ascontiguousarray(s["rest"], np.float32)
        self.k = np.ascontiguousarray(s["k"], np.float32)
        self.c = np.ascontiguousarray(s["c"], np.float32)
        self.flags = np.ascontiguousarray(s["flags"], np.uint8)
        self.minl = np.ascontiguousarray(s["minl"], np.float32)
        self.maxl = np.ascontiguousarray(s["maxl"], np.float32)
        self.stride = np.ascontiguousarray(s["stride"], np.float32)
        # muscle state starts at originx = the muscle edges' rest length
        idx = np.concatenate([np.arange(self.edge_off[w], self.edge_off[w] + self.n_muscles[w])
                              for w in range(self.N)]) if self.N else np.zeros(0, np.int64)
        mx = s.get("mx")
        self.mx = (self.rest[idx.astype(np.int64)].copy() if mx is None
                   else np.ascontiguousarray(mx, np.float32).copy())
        self.steps = np.zeros(self.N, np.int32) if s.get("steps") is None else \
            np.ascontiguousarray(s["steps"], np.int32).copy()
        self.contact = np.zeros(len(self.m), np.uint8)
        pin = s.get("pinned")
        self.pinned = None if pin is None or not np.any(pin) else np.ascontiguousarray(pin, np.uint8).copy()
        # Point.e / Point.r (gym/engine.py:31-50: e = Config.e, r = m ** 0.3 unless given), Python floats
        ch = s.get("charge")
        self.charge = None if ch is None else np.ascontiguousarray(ch, np.float64).copy()
        rad = s.get("radius")
        self.radius = (self.m.astype(np.float64) ** 0.3 if rad is None
                       else np.ascontiguousarray(rad, np.float64)).copy()
        bs = s.get("bounce_set")   # Point.bounce(k, other=<list>): bit 0 caller, bit 1 in the list (None: all, "*")
        self.bounce_set = None if bs is None else np.ascontiguousarray(bs, np.uint8).reshape(-1).copy()
        self.n_threads = n_threads
        Ms = np.diff(self.mass_off)
        d = 3 if P["in3d"] else 2
        self.obs_len = (3 * d * Ms + (3 if P["conmid"] else 0) + self.n_muscles).astype(np.int32)
        self.obs_stride = int(self.obs_len.max()) if self.N else 0
        self._mk_structs()

    def _mk_structs(self):
        P = self.params
        types = dict(OrcParams._fields_)
        self._params = OrcParams(**{k: (float(v) if types[k] is C.c_double else
                                        types[k](*[float(x) for x in v]) if k == "g3_gravity" else int(v))
                                    for k, v in P.items()})
        self._batch = OrcBatch(
            self.N, _p(self.mass_off, _i32p), _p(self.edge_off, _i32p), _p(self.muscle_off, _i32p),
            _p(self.pos, _f32p), _p(self.vel, _f32p), _p(self.acc, _f32p), _p(self.m, _f32p),
            _p(self.ei, _i32p), _p(self.ej, _i32p), _p(self.rest, _f32p), _p(self.k, _f32p),
            _p(self.c, _f32p), _p(self.flags, _u8p), _p(self.mx, _f32p), _p(self.minl, _f32p),
            _p(self.maxl, _f32p), _p(self.stride, _f32p), _p(self.steps, _i32p), _p(self.contact, _u8p),
            _p(self.pinned, _u8p), _p(self.charge, _f64p), _p(self.radius, _f64p), _p(self.bounce_set, _u8p))

    def set_params(self, **kw):
        """Change env parameters between steps (the state stays), as BatchedPhysicsEnv.set_params."""
        for k, v in kw.items():
            if k not in self.params:
                raise KeyError(k)
            self.params[k] = v
        self._mk_structs()

    def _outs(self):
        o = dict(obs=np.zeros((self.N, self.obs_stride), np.float32), reward=np.zeros(self.N, np.float32),
                 done=np.zeros(self.N, np.uint8), centroid=np.zeros((self.N, 3), np.float32),
                 energy=np.zeros(self.N, np.float32))
        s = OrcOut(_p(o["obs"], _f32p), self.obs_stride, _p(o["reward"], _f32p), _p(o["done"], _u8p),
                   _p(o["centroid"], _f32p), _p(o["energy"], _f32p))
        return o, s

    def step(self, action=None, observe=True):
        L = lib()
        act = None if action is None else np.ascontiguousarray(action, np.float32).reshape(self.N, -1)
        cols = 0 if act is None else act.shape[1]
        o, s = self._outs() if observe else (None, None)
        rc = L.orc_step(C.byref(self._batch), C.byref(self._params), _p(act, _f32p), cols, cols,
                        C.byref(s) if s is not None else None, self.n_threads)
        if rc != 0:
            raise RuntimeError(f"orc_step failed: {rc}")
        return o

    def observe(self):
        o, s = self._outs()
        lib().orc_observe(C.byref(self._batch), C.byref(self._params), C.byref(s), self.n_threads)
        return o

    def reset(self, noise=None):
        nz = None if noise is None else np.ascontiguousarray(noise, np.float32).reshape(-1, 3)
        lib().orc_reset(C.byref(self._batch), C.byref(self._params), _p(nz, _f32p), self.n_threads)
        return self.observe()


def np_norm3(v) -> float:
    v = np.ascontiguousarray(v, np.float32)
    return float(lib().orc_np_norm3(v.ctypes.data_as(_f32p)))


def np_pairwise_sum(a) -> float:
    a = np.ascontiguousarray(a, np.float32)
    return float(lib().orc_np_pairwise_sum(a.ctypes.data_as(_f32p), len(a), 1))


def spec_from_npz(z) -> tuple[dict, dict]:
    """Split a golden .npz into (spec dict, params dict)."""
    spec = {k[3:]: z[k] for k in z.files if k.startswith("in_")}
    params = {k[6:]: z[k].item() for k in z.files if k.startswith("param_")}
    params["action_mode"] = int(z["action_mode"])
    return spec, params


def momentum(vel, m, mass_off) -> np.ndarray:
    """Point.momentum of every walker (gym/engine.py:160-166): m_sum = zeros(3, float32), then m_sum += p.v * p.m
    point by point in point order — numpy's float32 product and float32 add, restated with float32 arrays (one
    sequential step per point index, vectorised across walkers)."""
    vel = np.asarray(vel, np.float32).reshape(-1, 3)
    m = np.asarray(m, np.float32)
    mass_off = np.asarray(mass_off, np.int64)
    N = len(mass_off) - 1
    Ms = np.diff(mass_off)
    out = np.zeros((N, 3), np.float32)
    for q in range(int(Ms.max()) if N else 0):
        sel = Ms > q
        idx = mass_off[:-1][sel] + q
        out[sel] = out[sel] + vel[idx] * m[idx][:, None]
    return out


def nonfinite(pos, vel, acc, mass_off) -> np.ndarray:
    """1 for a walker any of whose pos / vel / acc components is inf or NaN (SURVEY §5 failure detection)."""
    bad = ~(np.isfinite(np.asarray(pos).reshape(-1, 3)).all(1) & np.isfinite(np.asarray(vel).reshape(-1, 3)).all(1)
            & np.isfinite(np.asarray(acc).reshape(-1, 3)).all(1))
    mass_off = np.asarray(mass_off, np.int64)
    return np.array([bad[a:b].any() for a, b in zip(mass_off[:-1], mass_off[1:])], np.uint8)
