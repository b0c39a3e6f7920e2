"""Walker topology packer and HBM layout.

The reference keeps one Python object per mass (gym/engine.py:24-59) and per edge
(gym/optimized_walker.py:7-106).  Here a batch of walkers is flat structure-of-arrays in HBM,
ordered by walker so that any contiguous walker range is a contiguous byte range of every array:

  per mass   pos, vel, acc (old_a)  f32[P,3];  mass f32[P];  contact u8[P]
  per edge   edges: 16-B records {ij = i | j<<16 | string<<31 (walker-local), rest, k, c} [E]
  per walker-edge-end   inc u16[2E] = (edge<<1 | end) sorted by (mass, edge, end);
             inc_off u16[P+N] (M_w+1 offsets per walker) — the deterministic accumulation order
  per muscle muscle_x f32[U]; bounds (lo, hi) = (f32(originx*minl), f32(originx*maxl)) f32[U,2];
             stride f32[U] (discrete actions)
  per walker steps i32[N]
Muscles are the first A_w edges of each walker (Creature.run order, gym/optimized_walker.py:124-127).
Uniform batches (one M/K/A) carry no offsets; ragged ones carry CSR mass_off/edge_off/muscle_off.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import os

import numpy as np

f32 = np.float32
SPEC_KEYS = ("m", "pos", "vel", "mass_off", "ei", "ej", "rest", "k", "c", "flags", "edge_off", "n_muscles",
             "minl", "maxl", "stride")


@dataclass
class HostLayout:
    """Packed host arrays, ready to upload.  All arrays are C-contiguous numpy."""
    N: int
    M: int            # uniform: masses per walker; ragged: max
    K: int
    A: int
    ragged: bool
    mass_off: np.ndarray
    edge_off: np.ndarray
    muscle_off: np.ndarray
    pos: np.ndarray
    vel: np.ndarray
    acc: np.ndarray
    mass: np.ndarray
    edges: np.ndarray          # uint32 [E, 4]: ij (with string bit 31), rest, k, c (float bits)
    inc: np.ndarray
    inc_off: np.ndarray
    muscle_x: np.ndarray
    muscle_bounds: np.ndarray  # float32 [U, 2]
    muscle_stride: np.ndarray
    steps: np.ndarray
    pinned: Optional[np.ndarray] = None   # uint8 [P]: DingPoint masses (None = no pinned mass)
    charge: Optional[np.ndarray] = None   # float64 [P]: Point.e (None = Config.e for every point)
    radius: Optional[np.ndarray] = None   # float64 [P]: Point.r (None = m ** 0.3, gym/engine.py:45-46)
    # uint8 [P]: Point.bounce(k, other=<list>) (gym/engine.py:114-125): bit 0 = calls bounce, bit 1 = in the list
    # (None = every point calls, other="*")
    bounce_set: Optional[np.ndarray] = None
    # ragged batches are stored in wave-tile / size order (size_order): row [N] = the caller's index of each stored walker, mass_perm /
    # muscle_perm = the stored index of each caller mass / muscle (None = stored in the caller's order)
    row: Optional[np.ndarray] = None
    mass_perm: Optional[np.ndarray] = None
    muscle_perm: Optional[np.ndarray] = None
    extra: Dict[str, np.ndarray] = field(default_factory=dict)

    @property
    def P(self) -> int:
        return int(self.mass_off[-1])

    @property
    def E(self) -> int:
        return int(self.edge_off[-1])

    @property
    def U(self) -> int:
        return int(self.muscle_off[-1])

    def obs_len(self, in3d: bool, conmid: bool) -> np.ndarray:
        """Observation length of every walker, in the CALLER's order."""
        d = 3 if in3d else 2
        n = (3 * d * np.diff(self.mass_off) + (3 if conmid else 0) + np.diff(self.muscle_off)).astype(np.int32)
        if self.row is None:
            return n
        out = np.empty_like(n)
        out[self.row] = n
        return out


def incidence(ei: np.ndarray, ej: np.ndarray, mass_off: np.ndarray, edge_off: np.ndarray):
    """Per-walker incidence lists in reference accumulation order.

    For mass q of walker w the list holds (e<<1 | end) for every edge e of w with ei[e]==q (end 0) or
    ej[e]==q (end 1), sorted by e then end — the order in which gym/optimized_walker.py:124-127 +
    gym/engine.py:101-102 add spring/damping terms to q's acceleration.
    Returns inc u16[2E] (walker w's list at 2*edge_off[w]) and inc_off u16[P+N]
    (walker w's M_w+1 offsets at mass_off[w]+w, walker-local)."""
    N = len(mass_off) - 1
    Ks = np.diff(edge_off).astype(np.int64)
    Ms = np.diff(mass_off).astype(np.int64)
    E = int(edge_off[-1])
    if E and (Ks.max() * 2 > 65535):
        raise ValueError("a walker with more than 32767 edges does not fit the u16 incidence encoding")
    wid = np.repeat(np.arange(N, dtype=np.int64), Ks)
    local_e = np.arange(E, dtype=np.int64) - np.repeat(edge_off[:-1].astype(np.int64), Ks)
    # two entries per edge: (mass, edge, end)
    mass = np.stack([ei.astype(np.int64), ej.astype(np.int64)], 1).reshape(-1)
    end = np.tile(np.array([0, 1], np.int64), E)
    e2 = np.repeat(local_e, 2)
    w2 = np.repeat(wid, 2)
    if E and (mass.min() < 0 or np.any(mass >= np.repeat(Ms, 2 * Ks))):
        raise ValueError("edge endpoint out of range of its walker")
    maxk = int(Ks.max()) if N else 0
    key = ((w2 * (int(Ms.max()) + 1 if N else 1) + mass) * (2 * maxk + 2) + 2 * e2 + end)
    order = np.argsort(key, kind="stable")
    inc = ((e2[order] << 1) | end[order]).astype(np.uint16)
    # counts per (walker, mass) -> offsets
    counts = np.zeros(int(mass_off[-1]), np.int64)
    np.add.at(counts, np.repeat(mass_off[:-1].astype(np.int64), 2 * Ks) + mass, 1)
    inc_off = np.zeros(int(mass_off[-1]) + N, np.uint16)
    for_w = np.repeat(np.arange(N, dtype=np.int64), Ms)
    csum = np.cumsum(counts)
    start_w = np.concatenate([[0], csum])[mass_off[:-1].astype(np.int64)]   # global start of walker
    excl = np.concatenate([[0], csum[:-1]]) - start_w[for_w]                 # walker-local start of mass
    q_local = np.arange(int(mass_off[-1]), dtype=np.int64) - mass_off[:-1].astype(np.int64)[for_w]
    pos_in = mass_off[:-1].astype(np.int64)[for_w] + for_w + q_local
    inc_off[pos_in] = excl.astype(np.uint16)
    inc_off[(mass_off[1:].astype(np.int64) + np.arange(N))] = (2 * Ks).astype(np.uint16)
    return inc, inc_off


def pack(spec: Dict[str, np.ndarray], mx: Optional[np.ndarray] = None, steps: Optional[np.ndarray] = None,
         sort: bool = True) -> HostLayout:
    """Pack a flat CSR spec (see walker_gym_amd.synthetic) into the HBM layout.  A ragged batch is stored in
    size_order (``sort``; HostLayout.row / mass_perm / muscle_perm map it back to the caller's order)."""
    if mx is not None:
        spec = dict(spec, mx=mx)
    if steps is not None:
        spec = dict(spec, steps=steps)
    Ms, Ks = np.diff(np.asarray(spec["mass_off"])), np.diff(np.asarray(spec["edge_off"]))
    nm = np.asarray(spec["n_muscles"])
    uniform = len(Ms) > 0 and np.all(Ms == Ms[0]) and np.all(Ks == Ks[0]) and np.all(nm == nm[0])
    row = mass_perm = muscle_perm = None
    if sort and not uniform and len(Ms) > 1:
        order = size_order(spec)
        if np.any(order != np.arange(len(order))):
            spec = reorder_walkers(spec, order)
            if spec.get("steps") is not None:
                spec["steps"] = np.asarray(spec["steps"])[order]
            row, mass_perm, muscle_perm = order.astype(np.int32), spec["_mass_perm"], spec["_muscle_perm"]
    lay = _pack(spec, spec.get("mx"), spec.get("steps"))
    lay.row, lay.mass_perm, lay.muscle_perm = row, mass_perm, muscle_perm
    return lay


def _pack(spec: Dict[str, np.ndarray], mx: Optional[np.ndarray], steps: Optional[np.ndarray]) -> HostLayout:
    s = {k: np.asarray(spec[k]) for k in SPEC_KEYS}
    mass_off = np.ascontiguousarray(s["mass_off"], np.int32)
    edge_off = np.ascontiguousarray(s["edge_off"], np.int32)
    n_mus = np.ascontiguousarray(s["n_muscles"], np.int32)
    N = len(mass_off) - 1
    muscle_off = np.concatenate([[0], np.cumsum(n_mus)]).astype(np.int32)
    Ms, Ks = np.diff(mass_off), np.diff(edge_off)
    if N == 0:
        raise ValueError("empty batch")
    if np.any(Ms < 1):
        raise ValueError("every walker needs at least one mass")
    if np.any(n_mus > Ks):
        raise ValueError("a walker has more muscles than edges (muscles are the first edges)")
    if Ms.max() > 1024:
        raise ValueError("walkers with more than 1024 masses are not supported (WG_MAX_M)")
    ragged = not (np.all(Ms == Ms[0]) and np.all(Ks == Ks[0]) and np.all(n_mus == n_mus[0]))
    ei = np.ascontiguousarray(s["ei"], np.int64)
    ej = np.ascontiguousarray(s["ej"], np.int64)
    if Ms.max() > 32767:
        raise ValueError("walker-local mass index does not fit the 15-bit edge endpoint encoding")
    flags = np.ascontiguousarray(s["flags"], np.uint8)
    edge_ij = (ei.astype(np.uint32) | (ej.astype(np.uint32) << np.uint32(16))
               | ((flags & 1).astype(np.uint32) << np.uint32(31))).astype(np.uint32)
    inc, inc_off = incidence(ei, ej, mass_off, edge_off)
    rest = np.ascontiguousarray(s["rest"], f32)
    # muscle u of walker w is edge edge_off[w] + (u - muscle_off[w]); originx = its rest
    uw = np.repeat(np.arange(N), n_mus)
    medge = edge_off[:-1][uw] + (np.arange(int(muscle_off[-1])) - muscle_off[:-1][uw])
    x0 = rest[medge]
    minl = np.ascontiguousarray(s["minl"], f32)
    maxl = np.ascontiguousarray(s["maxl"], f32)
    # Muscle.regulation computes originx*minl / originx*maxl in float32 each call (optimized_walker.py:29-30)
    lo = (x0 * minl).astype(f32)
    hi = (x0 * maxl).astype(f32)
    pos = np.ascontiguousarray(s["pos"], f32).reshape(-1, 3)
    acc = spec.get("acc")
    edges = np.stack([edge_ij, rest.view(np.uint32), np.ascontiguousarray(s["k"], f32).view(np.uint32),
                      np.ascontiguousarray(s["c"], f32).view(np.uint32)], axis=1) if len(rest) else \
        np.zeros((0, 4), np.uint32)
    return HostLayout(
        N=N, M=int(Ms.max()), K=int(Ks.max()), A=int(n_mus.max()), ragged=bool(ragged),
        mass_off=mass_off, edge_off=edge_off, muscle_off=muscle_off,
        pos=pos.copy(), vel=np.ascontiguousarray(s["vel"], f32).reshape(-1, 3).copy(),
        acc=(np.zeros_like(pos) if acc is None else np.ascontiguousarray(acc, f32).reshape(-1, 3).copy()),
        mass=np.ascontiguousarray(s["m"], f32), edges=np.ascontiguousarray(edges, np.uint32),
        inc=inc, inc_off=inc_off,
        muscle_x=(x0.copy() if mx is None else np.ascontiguousarray(mx, f32).copy()),
        muscle_bounds=np.ascontiguousarray(np.stack([lo, hi], axis=1).reshape(-1, 2), f32),
        muscle_stride=np.ascontiguousarray(s["stride"], f32),
        steps=(np.zeros(N, np.int32) if steps is None else np.ascontiguousarray(steps, np.int32).copy()),
        pinned=_pinned(spec, int(mass_off[-1])),
        charge=_per_mass_f64(spec, "charge", int(mass_off[-1])),
        radius=_per_mass_f64(spec, "radius", int(mass_off[-1])),
        bounce_set=_bounce_set(spec, int(mass_off[-1])),
    )


def _per_mass_f64(spec, key: str, P: int):
    """Point.e / Point.r: Python floats in the reference, kept as float64."""
    a = spec.get(key)
    if a is None:
        return None
    a = np.ascontiguousarray(a, np.float64).reshape(-1)
    if a.shape[0] != P:
        raise ValueError(f"{key} has {a.shape[0]} entries for {P} masses")
    return a.copy()


def default_radius(mass: np.ndarray) -> np.ndarray:
    """Point.__init__ radius r = m ** 0.3 (gym/engine.py:45-46), m the stored float32 mass as a Python float."""
    return np.asarray(mass, np.float32).astype(np.float64) ** 0.3


def bounce_set_from_lists(n_points: int, callers, other="*") -> np.ndarray:
    """One walker's `bounce_set` bytes from the reference's calls `for p in callers: p.bounce(k, other=other)`
    (gym/engine.py:114-126), as point indices of the walker.  The two-bit encoding holds exactly this: the callers in
    registry order (ascending, each once) and ONE `other` list shared by every caller, in registry order (ascending,
    each once; "*" = every point).  The reference iterates `other` in the order given and float32 accumulation
    follows that order, so a list in any other order, with a repeated point, or different per caller changes the
    reference's bits and is not expressible: it raises ValueError instead of silently reordering."""
    def idx(lst, what):
        a = np.asarray(list(lst), np.int64).reshape(-1)
        if a.size and (a.min() < 0 or a.max() >= n_points):
            raise ValueError(f"bounce {what}: point index out of range [0, {n_points})")
        if a.size > 1 and not bool(np.all(np.diff(a) > 0)):
            raise ValueError(f"bounce {what} must be in registry order (ascending point indices, no repeats): the "
                             "reference iterates the list as given, which bounce_set cannot express otherwise")
        return a
    bs = np.zeros(n_points, np.uint8)
    bs[idx(callers, "callers")] |= 1
    if isinstance(other, str):
        if other != "*":
            raise ValueError('bounce other must be "*" or a list of point indices')
        bs |= 2
    else:
        bs[idx(other, "other")] |= 2
    return bs


def _bounce_set(spec, P: int):
    """Per point, which side of Point.bounce(k, other=<list>) it is on: bit 0 the point calls bounce (callers in
    registry order), bit 1 it is in `other` (the list in registry order); other bits must be 0.  All 3 is the
    reference's default other="*" and is stored as None.  Restriction: one shared `other` list per walker, iterated in
    registry order (bounce_set_from_lists builds the bytes and rejects what they cannot express)."""
    bs = spec.get("bounce_set")
    if bs is None:
        return None
    bs = np.ascontiguousarray(bs).reshape(-1)
    if bs.shape[0] != P:
        raise ValueError(f"bounce_set has {bs.shape[0]} entries for {P} masses")
    if bs.size and (bs.min() < 0 or bs.max() > 3):
        raise ValueError("bounce_set entries are bit 0 (calls bounce) | bit 1 (in the other list): 0..3")
    bs = bs.astype(np.uint8)
    return None if bool(np.all(bs == 3)) else bs.copy()


def _pinned(spec, P: int):
    pin = spec.get("pinned")
    if pin is None:
        return None
    pin = np.ascontiguousarray(pin, np.uint8).reshape(-1)
    if pin.shape[0] != P:
        raise ValueError(f"pinned has {pin.shape[0]} entries for {P} masses")
    return (pin != 0).astype(np.uint8) if pin.any() else None


def reorder_walkers(spec: Dict[str, np.ndarray], order: np.ndarray) -> Dict[str, np.ndarray]:
    """The flat CSR spec with its walkers in ``order`` (stored walker w = spec walker order[w])."""
    order = np.asarray(order, np.int64)
    mo, eo = np.asarray(spec["mass_off"], np.int64), np.asarray(spec["edge_off"], np.int64)
    nm = np.asarray(spec["n_muscles"], np.int64)
    uo = np.concatenate([[0], np.cumsum(nm)])

    def gather(off):
        lens = np.diff(off)[order]
        starts = off[:-1][order]
        idx = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(int(lens.sum()))
        return idx, np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)

    pidx, new_mo = gather(mo)
    eidx, new_eo = gather(eo)
    uidx, _ = gather(uo)
    out = dict(spec)
    for k in ("m", "pos", "vel", "acc", "pinned", "charge", "radius", "bounce_set"):
        if spec.get(k) is not None:
            out[k] = np.asarray(spec[k])[pidx]
    for k in ("ei", "ej", "rest", "k", "c", "flags"):
        out[k] = np.asarray(spec[k])[eidx]
    for k in ("minl", "maxl", "stride", "mx"):
        if spec.get(k) is not None:
            out[k] = np.asarray(spec[k])[uidx]
    out["mass_off"], out["edge_off"] = new_mo, new_eo
    out["n_muscles"] = nm[order].astype(np.int32)
    out["_mass_perm"] = np.empty(len(pidx), np.int64)
    out["_mass_perm"][pidx] = np.arange(len(pidx))       # caller mass -> stored mass
    out["_muscle_perm"] = np.empty(len(uidx), np.int64)
    out["_muscle_perm"][uidx] = np.arange(len(uidx))
    return out


WAVE_LANES = 64          # masses / muscles per wave tile (walker_hip.hip walker_step_waves)
WAVE_MAX_WALKERS = 32    # walkers per wave tile (walker_hip.hip RW_MAXW)


def wave_edge_passes(M: int, K: int) -> int:
    """walker_hip.hip wave_passes (exported as wg_wave_edge_passes): spring passes of a wave tile for batch maxima
    M, K; 0 = the batch cannot use the wave kernel."""
    if M < 1 or M > 64 or K < 0:
        return 0
    ne = max((K + 63) // 64, (K + M - 1) // M, 1)
    return 0 if ne > 8 else (ne if ne <= 4 else 8)


def wave_tile_order(M: np.ndarray, K: np.ndarray, A: np.ndarray, ne: int, window: Optional[int] = None) -> np.ndarray:
    """Best-fit decreasing wave tiles (wave_tile_order_bfd) within windows of `window` consecutive CALLER walkers
    (default WG_TILE_WINDOW or 512), the windows in caller order.  A window's tiles are then consecutive wave tiles:
    with the kernel's XCD-aware workgroup order they run on one XCD, so the caller-order rows they scatter into
    (actions in; reward / done / centroid / energy / obs rows out) are fetched and merged in one L2 instead of being
    written back as partial lines from every XCD.  Config 5: 18,531 tiles at 512 against 18,469 for one global
    packing (+0.3 %).  window <= 0: one global packing."""
    if window is None:
        window = int(os.environ.get("WG_TILE_WINDOW", "512"))
    n = len(M)
    if window <= 0 or window >= n:
        return wave_tile_order_bfd(M, K, A, ne)
    parts = []
    for s in range(0, n, window):
        idx = np.arange(s, min(s + window, n))
        parts.append(idx[wave_tile_order_bfd(M[idx], K[idx], A[idx], ne)])
    return np.concatenate(parts)


def wave_tile_order_bfd(M: np.ndarray, K: np.ndarray, A: np.ndarray, ne: int) -> np.ndarray:
    """Best-fit decreasing packing of walkers into wave tiles (<= 64 masses, <= 64*ne springs, <= 64 muscles,
    <= 32 walkers), returned as a walker order with each tile's walkers contiguous: walkers largest first (masses,
    then springs, then muscles), each into the open tile with the fewest free mass lanes that still takes it.
    wg_plan_waves' greedy contiguous packing over this order gives exactly these tiles (a tile is opened only by a
    walker no earlier tile could take, and tiles only fill up).  Against tiles of size-sorted neighbours this fills
    the lanes: SURVEY §8(d)'s config 5 (M ~ U{4..32}) goes from 21,096 tiles (55.8 masses each) to 18,469 (63.7)."""
    n = len(M)
    order = np.lexsort((np.arange(n), -A, -K, -M))
    cap_e = WAVE_LANES * ne
    tiles = []                                   # [masses, springs, muscles, walkers, members]
    free = [[] for _ in range(WAVE_LANES + 1)]   # free mass lanes -> open tiles (most recent last)
    for w in order.tolist():
        m, k, a = int(M[w]), int(K[w]), int(A[w])
        placed = False
        for r in range(m, WAVE_LANES + 1):
            lst = free[r]
            for j in range(len(lst) - 1, -1, -1):
                t = tiles[lst[j]]
                if t[1] + k <= cap_e and t[2] + a <= WAVE_LANES and t[3] < WAVE_MAX_WALKERS:
                    ti = lst.pop(j)
                    t[0] += m; t[1] += k; t[2] += a; t[3] += 1; t[4].append(w)
                    free[WAVE_LANES - t[0]].append(ti)
                    placed = True
                    break
            if placed:
                break
        if not placed:
            tiles.append([m, k, a, 1, [w]])
            free[WAVE_LANES - m].append(len(tiles) - 1)
    return np.fromiter((w for t in tiles for w in t[4]), np.int64, n)


def size_order(spec: Dict[str, np.ndarray]) -> np.ndarray:
    """The stored order of a ragged batch ("sort by bucket").  Batches whose walkers all fit
    one wave (the wave kernel): wave_tile_order, each wave tile's walkers contiguous.  Otherwise (the workgroup
    kernel) walkers sorted by (masses, springs, muscles), stable, so that workgroup tiles pack evenly."""
    M = np.diff(np.asarray(spec["mass_off"], np.int64))
    K = np.diff(np.asarray(spec["edge_off"], np.int64))
    A = np.asarray(spec["n_muscles"], np.int64)
    if len(M):
        ne = wave_edge_passes(int(max(1, M.max())), int(K.max()))
        # WG_TILE_ORDER=sorted (diagnostic): size-sorted neighbours, the order before wave_tile_order
        if ne and int(A.max()) <= WAVE_LANES and os.environ.get("WG_TILE_ORDER", "bfd") != "sorted":
            return wave_tile_order(M, K, A, ne)
    return np.lexsort((np.arange(len(M)), A, K, M))


def algorithmic_bytes_per_walker_step(M: int, K: int, A: int, obs_floats: int) -> int:
    """B = 64M + 16K + 20A + 8 (+ 4 per materialised obs float)."""
    return 64 * M + 16 * K + 20 * A + 8 + 4 * obs_floats


def layout_bytes_per_walker_step(M, K, A, obs_floats, info: bool = True, contact: bool = True,
                                 ragged: bool = False):
    """Bytes THIS layout moves per walker-step (the survey's B plus what the layout adds):
    incidence lists u16[2K] + offsets u16[M+1], centroid/energy (16 B) and contact (M B); the muscle
    edges' unused rest entries are not read (-4A).  Ragged batches (the wave kernel) also read the walker's CSR
    offsets (mass_off / edge_off / muscle_off, 12 B) and its caller row (row, 4 B).  Scalars or per-walker arrays."""
    b = algorithmic_bytes_per_walker_step(M, K, A, obs_floats)
    b = b + 2 * 2 * K + 2 * (M + 1) - 4 * A
    if info:
        b = b + 16
    if contact:
        b = b + M
    if ragged:
        b = b + 16
    return b
