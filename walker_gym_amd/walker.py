"""Muscle / Skeleton / Creature and the reference topologies, as builders of packed batches.

Mirrors gym/optimized_walker.py:7-224: element constructors keep the reference's argument names and
defaults (k=1000, maxl=1.5, minl=0.1, stride=2, dampk=20); a rest length ``x=None`` is the current
distance computed with the same ``np.linalg.norm`` call (gym/optimized_walker.py:23-25, 80-82).
``creatures_to_spec`` packs a list of creatures into the flat CSR spec the env consumes: muscles first,
then skeletons, in list order (Creature.run order, :124-127).
"""
from __future__ import annotations

from typing import List

import numpy as np

from .engine import DingPoint, Point

f32 = np.float32


class Muscle:
    """Actuated spring (gym/optimized_walker.py:7-67)."""

    def __init__(self, p1: Point, p2: Point, x: float = None, k: float = 1000, maxl: float = 1.5,
                 minl: float = 0.1, stride: float = 2, dampk: float = 20, string: bool = False):
        self.p1, self.p2 = p1, p2
        self.x = self.distant(p1, p2) if x is None else x
        self.originx = self.x
        self.k, self.dampk = k, dampk
        self.minl, self.maxl, self.stride = minl, maxl, stride
        self.string = string

    @staticmethod
    def distant(p1: Point, p2: Point) -> float:
        return np.linalg.norm(p1.pos - p2.pos)

    def regulation(self) -> None:
        self.x = max(self.x, self.originx * self.minl)
        self.x = min(self.x, self.originx * self.maxl)

    def act(self, a: float) -> None:
        self.x += a
        self.regulation()

    def actdisp(self, a: bool) -> None:
        self.x = self.x + self.stride if a else self.x - self.stride
        self.regulation()


class Skeleton:
    """Passive spring (gym/optimized_walker.py:69-106); ``string=True`` is engine.py's rope mode
    (gym/engine.py:97-98: no force while compressed)."""

    def __init__(self, p1: Point, p2: Point, x: float = None, k: float = 1000, dampk: float = 20,
                 string: bool = False):
        self.p1, self.p2 = p1, p2
        self.x = Muscle.distant(p1, p2) if x is None else x
        self.k, self.dampk = k, dampk
        self.string = string


class Creature:
    """gym/optimized_walker.py:108-172.  Physics runs batched in the env; ``act``/``actdisp`` update
    the host-side description before packing (after packing, use the env's ``step``)."""

    def __init__(self, phylist: List[Point], musclelist: List[Muscle], skeletonlist: List[Skeleton]):
        self.phys = phylist
        self.muscles = musclelist
        self.skeletons = skeletonlist

    def act(self, a) -> None:
        for i in range(min(len(self.muscles), len(a))):
            self.muscles[i].act(a[i])

    def actdisp(self, a) -> None:
        for i in range(min(len(self.muscles), len(a))):
            self.muscles[i].actdisp(a[i])


def create_balance_creature() -> Creature:
    """gym/optimized_walker.py:176-199 (Balance-v0)."""
    p = [Point(5, [-50, 100, 0], [0, 0, 0]), Point(5, [50, 100, 0], [0, 0, 0]),
         Point(1, [0, 0, 0], [0, 0, 0]), Point(3, [0, 100, 0], [0, 0, 0])]
    sk = [Skeleton(p[0], p[1]), Skeleton(p[0], p[3]), Skeleton(p[1], p[3])]
    m = [Muscle(p[0], p[2]), Muscle(p[1], p[2])]
    return Creature(p, m, sk)


def create_box_creature() -> Creature:
    """gym/optimized_walker.py:201-224 (Box-v0)."""
    p = [Point(1, [-50, 0, 0], [0, 0, 0]), Point(1, [-50, 100, 0], [0, 0, 0]),
         Point(1, [50, 100, 0], [0, 0, 0]), Point(1, [50, 0, 0], [0, 0, 0])]
    sk = [Skeleton(p[1], p[2])]
    m = [Muscle(p[0], p[1]), Muscle(p[0], p[2]), Muscle(p[3], p[1]), Muscle(p[3], p[2])]
    return Creature(p, m, sk)


def creatures_to_spec(creatures: List[Creature]) -> dict:
    """Pack creatures (each with its own points) into the flat CSR spec."""
    m, pos, vel, acc, mass_off = [], [], [], [], [0]
    ei, ej, rest, k, c, flags, edge_off = [], [], [], [], [], [], [0]
    nmus, minl, maxl, stride, mx, pinned = [], [], [], [], [], []
    charge, radius = [], []   # Point.e / Point.r (gym/engine.py:31-50), Python floats: pair_mode coulomb / bounce
    for cr in creatures:
        local = {}
        for p in cr.phys:
            if id(p) in local:
                raise ValueError("a point appears twice in one creature")
            local[id(p)] = len(local)
            m.append(float(p.m)); pos.append(np.asarray(p.pos, f32)); vel.append(np.asarray(p.v, f32))
            acc.append(np.asarray(p.old_a, f32))
            pinned.append(1 if isinstance(p, DingPoint) else 0)
            charge.append(float(getattr(p, "e", 16e-20))); radius.append(float(getattr(p, "r", float(p.m) ** 0.3)))
        mass_off.append(len(m))
        for e in list(cr.muscles) + list(cr.skeletons):
            if id(e.p1) not in local or id(e.p2) not in local:
                raise ValueError("an element references a point outside its creature")
            ei.append(local[id(e.p1)]); ej.append(local[id(e.p2)])
            k.append(e.k); c.append(e.dampk); flags.append(1 if getattr(e, "string", False) else 0)
            rest.append(e.originx if isinstance(e, Muscle) else e.x)
        for mu in cr.muscles:
            minl.append(mu.minl); maxl.append(mu.maxl); stride.append(mu.stride); mx.append(mu.x)
        nmus.append(len(cr.muscles))
        edge_off.append(len(ei))
    P = len(m)
    return dict(m=np.array(m, f32), pos=np.array(pos, f32).reshape(P, 3), vel=np.array(vel, f32).reshape(P, 3),
                acc=np.array(acc, f32).reshape(P, 3), mass_off=np.array(mass_off, np.int32),
                ei=np.array(ei, np.int32), ej=np.array(ej, np.int32), rest=np.array(rest, f32),
                k=np.array(k, f32), c=np.array(c, f32), flags=np.array(flags, np.uint8),
                edge_off=np.array(edge_off, np.int32), n_muscles=np.array(nmus, np.int32),
                minl=np.array(minl, f32), maxl=np.array(maxl, f32), stride=np.array(stride, f32),
                mx=np.array(mx, f32), pinned=np.array(pinned, np.uint8),
                charge=np.array(charge, np.float64), radius=np.array(radius, np.float64))


def replicate_spec(spec: dict, n: int) -> dict:
    """n copies of a single-walker spec (vectorised; used for the 4,096-walker Balance config)."""
    N0 = len(spec["mass_off"]) - 1
    if N0 != 1:
        raise ValueError("replicate_spec expects a single walker")
    out = {}
    for key in ("m", "pos", "vel", "acc", "ei", "ej", "rest", "k", "c", "flags", "minl", "maxl", "stride", "mx",
                "pinned", "charge", "radius", "bounce_set"):
        if key in spec:
            a = np.asarray(spec[key])
            out[key] = np.tile(a, (n,) + (1,) * (a.ndim - 1))
    M = int(spec["mass_off"][1]); K = int(spec["edge_off"][1])
    out["mass_off"] = (np.arange(n + 1) * M).astype(np.int32)
    out["edge_off"] = (np.arange(n + 1) * K).astype(np.int32)
    out["n_muscles"] = np.repeat(np.asarray(spec["n_muscles"], np.int32), n)
    return out


def concat_specs(specs: List[dict]) -> dict:
    """Walkers of several flat CSR specs, in order, as one spec (offsets rebased)."""
    out = {}
    per = ("m", "pos", "vel", "acc", "ei", "ej", "rest", "k", "c", "flags", "minl", "maxl", "stride", "mx",
           "pinned", "charge", "radius", "bounce_set", "n_muscles")
    for key in per:
        parts = [np.asarray(s[key]) for s in specs if key in s]
        if len(parts) == len(specs):
            out[key] = np.concatenate(parts)
        elif parts:
            raise ValueError(f"concat_specs: '{key}' present in some specs only")
    for key in ("mass_off", "edge_off"):
        offs, base = [np.zeros(1, np.int32)], 0
        for s in specs:
            o = np.asarray(s[key], np.int64)
            offs.append((o[1:] + base).astype(np.int32))
            base += int(o[-1])
        out[key] = np.concatenate(offs)
    return out


def balance_spec(n: int = 1) -> dict:
    return replicate_spec(creatures_to_spec([create_balance_creature()]), n)


def box_spec(n: int = 1) -> dict:
    return replicate_spec(creatures_to_spec([create_box_creature()]), n)
