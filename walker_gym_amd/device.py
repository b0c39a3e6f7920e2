"""Device-resident walker batch: the HostLayout uploaded to PyTorch-ROCm tensors in HBM, plus the
ctypes structs handed to libwalker_hip.so.  PyTorch is plumbing here (allocation, streams,
torch.distributed); all per-step compute is the HIP kernel."""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np
import torch

from . import _lib
from .layout import HostLayout, default_radius


def _to_dev(a: np.ndarray, device) -> torch.Tensor:
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint16:
        t = torch.from_numpy(a.view(np.int16))
    elif a.dtype == np.uint32:
        t = torch.from_numpy(a.view(np.int32))
    else:
        t = torch.from_numpy(a)
    return t.to(device, non_blocking=False).contiguous()


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


class DeviceBatch:
    """All walker arrays as device tensors (owned here, borrowed by the kernel per launch)."""

    STATE = ("pos", "vel", "acc", "muscle_x", "steps")   # + radius when kept (Point.bounce)

    def __init__(self, host: HostLayout, device: torch.device, contact: bool = True, wave_ok: bool = True):
        if device.type != "cuda":
            raise ValueError("DeviceBatch needs a ROCm device (torch 'cuda' device); there is no CPU path")
        self.host = host
        self.device = device
        self.N, self.M, self.K, self.A, self.ragged = host.N, host.M, host.K, host.A, host.ragged
        self.P, self.E, self.U = host.P, host.E, host.U
        dv = device
        self.mass_off = _to_dev(host.mass_off, dv)
        self.edge_off = _to_dev(host.edge_off, dv)
        self.muscle_off = _to_dev(host.muscle_off, dv)
        self.pos = _to_dev(host.pos, dv)
        self.vel = _to_dev(host.vel, dv)
        self.acc = _to_dev(host.acc, dv)
        self.mass = _to_dev(host.mass, dv)
        self.edges = _to_dev(host.edges, dv)
        self.inc = _to_dev(host.inc, dv) if host.E else None
        self.inc_off = _to_dev(host.inc_off, dv)
        self.muscle_x = _to_dev(host.muscle_x, dv)
        self.muscle_bounds = _to_dev(host.muscle_bounds, dv)
        self.muscle_stride = _to_dev(host.muscle_stride, dv)
        self.steps = _to_dev(host.steps, dv)
        self.contact = torch.zeros(self.P, dtype=torch.uint8, device=dv) if contact else None
        self.pinned = _to_dev(host.pinned, dv) if host.pinned is not None else None
        self.charge = _to_dev(host.charge, dv) if host.charge is not None else None
        self.bounce_set = _to_dev(host.bounce_set, dv) if host.bounce_set is not None else None
        self.radius = None   # allocated by enable_radius(): the step writes it, so only when bounce needs it
        # placeholders so that zero-size arrays still have a valid device pointer
        self._dummy = torch.zeros(16, dtype=torch.float32, device=dv)
        # ragged batches are stored in wave-tile / size order (layout.pack): row = caller index of each stored walker
        self.row = _to_dev(host.row, dv) if host.row is not None else None
        self._perm = {}
        if host.row is not None:
            inv = np.empty(self.N, np.int64)
            inv[host.row] = np.arange(self.N)
            self._perm = {"walker": torch.from_numpy(inv).to(dv), "row": torch.from_numpy(host.row.astype(np.int64)).to(dv),
                          "mass": torch.from_numpy(host.mass_perm).to(dv),
                          "muscle": torch.from_numpy(host.muscle_perm).to(dv)}
        self.plan = None
        self.plan_blocks = 0
        self.ragged_kind = 0
        self.version = 0   # bumped by every host-side write of the state (load_state_dict, setters, reset)
        self.replan(wave_ok)

    def replan(self, wave_ok: bool) -> None:
        """Choose the launch plan for parameters that can (wave_ok) or cannot use the barrier-free wave kernel.
        wave_ok (spring_mode 0, no pair forces): a uniform batch the lean kernel does not take (M not dividing 64)
        becomes wave tiles of whole walkers (identity order), a ragged batch whose walkers each fit one wave gets
        wave tiles.  Otherwise the workgroup kernel runs, on its own plan: uniform workgroup tiles (uniform_geo packs
        e.g. 19 M = 13 walkers per 256 lanes) or wg_plan_ragged tiles — a wave plan would leave it at most 64 masses
        per workgroup, 3/4 of the lanes idle (pair forces, the G2 element, the G3 engine)."""
        host, L = self.host, _lib.load()
        self.wave_ok = bool(wave_ok)
        lean_shape = 4 <= self.M <= 64 and 64 % self.M == 0
        self.ragged = host.ragged
        self.plan, self.plan_host, self.plan_blocks, self.ragged_kind = None, None, 0, 0
        waves = (wave_ok and self.A <= 64 and L.wg_wave_edge_passes(self.M, self.K) > 0
                 and os.environ.get("WG_LEAN", "1") != "0")
        if (not self.ragged and not lean_shape and waves and os.environ.get("WG_UNIFORM_WAVES", "1") != "0"):
            # a uniform batch the lean kernel does not take (M not dividing 64): stepped as wave tiles of whole
            # walkers (the barrier-free wave kernel; identity order) instead of workgroup tiles
            self.ragged = True
        if self.ragged:
            plan = np.zeros(self.N + 1, np.int32)
            args = (host.mass_off.ctypes.data_as(C.c_void_p), host.edge_off.ctypes.data_as(C.c_void_p),
                    host.muscle_off.ctypes.data_as(C.c_void_p), self.N, plan.ctypes.data_as(C.c_void_p), self.N + 1)
            # wave tiles when every walker fits one wave (the wave kernel), workgroup tiles otherwise
            if waves:
                nb, self.ragged_kind = _lib.check(L.wg_plan_waves(*args), "wg_plan_waves"), 2
            else:
                nb, self.ragged_kind = _lib.check(L.wg_plan_ragged(*args), "wg_plan_ragged"), 1
            self.plan = _to_dev(plan[:nb + 1], self.device)
            self.plan_host = plan[:nb + 1].copy()   # block -> first stored walker (walker ranges of plan slices)
            self.plan_blocks = nb
        self.struct = self._make_struct()

    # ---- the caller's order (ragged batches are stored in wave-tile / size order; uniform batches are not permuted)
    def caller(self, name: str) -> torch.Tensor:
        """A state tensor in the caller's walker / mass / muscle order: the tensor itself for an unpermuted batch
        (a live, writable view), a gathered copy for a sorted ragged batch."""
        t = getattr(self, name)
        if t is None or not self._perm:
            return t
        return t.index_select(0, self._perm[self.KIND[name]])

    def stored_mass(self, q: int) -> int:
        """Stored index of the caller's mass q."""
        return int(self.host.mass_perm[q]) if self._perm else int(q)

    def to_stored(self, kind: str, t: torch.Tensor) -> torch.Tensor:
        """A per-mass ('mass'), per-muscle ('muscle') or per-walker ('walker') caller-order tensor in the stored order."""
        if not self._perm:
            return t
        if kind == "walker":
            return t.index_select(0, self._perm["row"])
        if kind not in ("mass", "muscle"):
            raise ValueError(f"to_stored: kind must be 'mass', 'muscle' or 'walker', not {kind!r}")
        out = torch.empty_like(t)
        out.index_copy_(0, self._perm[kind], t)
        return out

    def enable_radius(self) -> None:
        """Keep Point.r on the device (pair_mode & 4, Point.bounce): the spec's radii or m ** 0.3."""
        if self.radius is None:
            r = self.host.radius if self.host.radius is not None else default_radius(self.host.mass)
            self.radius = _to_dev(r, self.device)
            self.struct = self._make_struct()

    def _p(self, t):
        if t is None:
            return None
        if t.numel() == 0:
            return C.c_void_p(self._dummy.data_ptr())
        return C.c_void_p(t.data_ptr())

    def _make_struct(self) -> _lib.WgBatch:
        r = self.ragged
        return _lib.WgBatch(
            N=self.N, M=self.M, K=self.K, A=self.A, ragged=self.ragged_kind if r else 0, row=self._p(self.row),
            mass_off=self._p(self.mass_off) if r else None, edge_off=self._p(self.edge_off) if r else None,
            muscle_off=self._p(self.muscle_off) if r else None,
            pos=self._p(self.pos), vel=self._p(self.vel), acc=self._p(self.acc), mass=self._p(self.mass),
            edges=self._p(self.edges),
            inc=self._p(self.inc) if self.inc is not None else None, inc_off=self._p(self.inc_off),
            muscle_x=self._p(self.muscle_x), muscle_bounds=self._p(self.muscle_bounds),
            muscle_stride=self._p(self.muscle_stride), steps=self._p(self.steps), contact=self._p(self.contact),
            pinned=self._p(self.pinned), charge=self._p(self.charge), radius=self._p(self.radius),
            bounce_set=self._p(self.bounce_set))

    def sub_struct(self, w0: int, w1: int) -> _lib.WgBatch:
        """A WgBatch view of walkers [w0, w1) of a uniform batch: the same device memory, pointers offset
        (every array is walker-major).  Used to run disjoint walker ranges on separate streams."""
        if self.ragged:
            raise ValueError("sub_struct: uniform batches only")
        if not 0 <= w0 < w1 <= self.N:
            raise ValueError(f"sub_struct: bad walker range [{w0}, {w1})")
        M, K, A = self.M, self.K, self.A

        def off(t, elems):
            return None if t is None else C.c_void_p(t.data_ptr() + elems * t.element_size())

        return _lib.WgBatch(
            N=w1 - w0, M=M, K=K, A=A, ragged=0, mass_off=None, edge_off=None, muscle_off=None,
            pos=off(self.pos, 3 * M * w0), vel=off(self.vel, 3 * M * w0), acc=off(self.acc, 3 * M * w0),
            mass=off(self.mass, M * w0), edges=off(self.edges, 4 * K * w0),
            inc=off(self.inc, 2 * K * w0) if self.inc is not None else None,
            inc_off=off(self.inc_off, (M + 1) * w0),
            muscle_x=self._p(self.muscle_x) if A == 0 else off(self.muscle_x, A * w0),
            muscle_bounds=self._p(self.muscle_bounds) if A == 0 else off(self.muscle_bounds, 2 * A * w0),
            muscle_stride=self._p(self.muscle_stride) if A == 0 else off(self.muscle_stride, A * w0),
            steps=off(self.steps, w0), contact=off(self.contact, M * w0), pinned=off(self.pinned, M * w0),
            charge=off(self.charge, M * w0), radius=off(self.radius, M * w0), row=None,
            bounce_set=off(self.bounce_set, M * w0))

    def launch_geometry(self) -> dict:
        info = _lib.WgLaunchInfo()
        _lib.check(_lib.load().wg_launch_geometry(C.byref(self.struct), C.byref(info)), "wg_launch_geometry")
        # ragged batches: the plan's blocks (workgroup kernel) or wave tiles (wave kernel, waves per workgroup)
        blocks = info.blocks
        if self.ragged:
            wpb = max(1, info.threads // 64)
            blocks = -(-self.plan_blocks // wpb) if self.ragged_kind == 2 else self.plan_blocks
        geo = dict(threads=info.threads, walkers_per_block=info.walkers_per_block, blocks=blocks,
                   lds_bytes=info.lds_bytes)
        if self.ragged_kind == 2:
            geo["wave_tiles"] = self.plan_blocks
        return geo

    KIND = {"pos": "mass", "vel": "mass", "acc": "mass", "contact": "mass", "radius": "mass", "muscle_x": "muscle",
            "steps": "walker"}

    def state_dict(self) -> dict:
        """The walker state in the CALLER's walker / mass / muscle order, whatever order the batch is stored in (a
        ragged batch is stored in wave-tile or size order, which depends on the batch and on WG_TILE_ORDER): a dict
        saved under one storage order loads correctly under another."""
        sd = {k: self.caller(k).clone() for k in self.STATE}
        if self.radius is not None:
            sd["radius"] = self.caller("radius").clone()
        return sd

    def load_state_dict(self, sd: dict) -> None:
        """Inverse of state_dict: caller-order tensors copied into the stored order."""
        self.version += 1
        for k in self.STATE:
            getattr(self, k).copy_(self.to_stored(self.KIND[k], sd[k].to(self.device)))
        if "radius" in sd:
            self.enable_radius()
            self.radius.copy_(self.to_stored("mass", sd["radius"].to(self.device)))
