"""Topology import: the reference's creature builders packed for the stepper.

Three generations of builders live in the reference.  Each becomes the flat CSR spec of
``walker.creatures_to_spec`` (masses, positions, springs with rest / k / c / string flag, muscles first in
Creature.run order, pinned DingPoints), so any of them steps on the same kernels:

* **G1** ``gym/walker.py:138-353`` — leg2, box, box2, balance, balance2, balance3, intrian, humanb, insect,
  box4, leg, hat.  They are written against the pre-``Point`` constructor ``Phy(m, v, p)`` (mass,
  VELOCITY, position: the order gym/engine.py:570's DingPoint keeps), which the reference no longer
  defines.  ``Phy`` / ``G1DingPoint`` restore that constructor, and the G1 elements keep
  gym/walker.py's own default rest length ``distant`` (:4-5: float32 ``**`` arithmetic, not
  ``np.linalg.norm``), so a packed G1 creature is bit-identical to the reference builder's
  (tests/golden/g1_builders.npz, generated from gym/walker.py itself).  Observe G1 creatures with
  ``midform=2``: G1 ``Creature.getstat`` (:83-101) subtracts the SUM of the positions.
* **G2** ``gym/optimized_walker.py:176-224`` — Balance-v0 / Box-v0 (``walker.create_*_creature``).
* **G3** ``gym/optimized_walker/walker.py:377-639`` — leg2, box, balance1..3, humanb, insect(legs).  G3's
  own physics (sinusoid CPG muscles, position-clamp ground, gym/optimized_walker/env.py:135-184) is out of
  scope.  What is imported is the geometry: masses, positions, pinned ``is_ding``
  points, springs (``k``, rest ``x``, ``string``; G3 default k = 100, env.py:92-111) as skeletons, and
  muscles as actuated springs of stiffness ``power`` and rest ``x`` (``np.linalg.norm(...)`` in float32
  when None, gym/optimized_walker/walker.py:29-33), damped with ``spring_dampk`` (the G2 default 20).
  tests/golden/g3_builders.npz holds the reference builders' own points and springs.

``topology_spec(name, n, generation)`` replicates one creature ``n`` times (uniform batch);
``mixed_spec([(name, count), ...])`` builds a ragged batch.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List

import numpy as np

from .engine import DingPoint, Point
from .walker import (Creature, Muscle, Skeleton, create_balance_creature, create_box_creature, creatures_to_spec,
                     replicate_spec)


# ---------------------------------------------------------------------------------------------- G1
def Phy(m: float, v, p, r: float = None, color="black") -> Point:
    """The G1 point constructor ``Phy(m, v, p)`` gym/walker.py calls (velocity before position)."""
    return Point(m, p, v, r, color)


def G1DingPoint(m: float, v, p, r: float = None, color="black") -> DingPoint:
    """gym/engine.py:569-579 ``DingPoint(m, v, p)``: a pinned point, G1 argument order."""
    return DingPoint(m, p, v, r, color)


def g1_distant(p1: Point, p2: Point):
    """gym/walker.py:4-5 on the float32 coordinates: ((dx**2 + dy**2 + dz**2) ** 0.5), numpy float32
    scalar arithmetic throughout (``**`` is powf), which can differ from np.linalg.norm in the last bit."""
    a, b = p1.pos, p2.pos
    return ((a[0] - b[0]) ** 2 + (a[1] - b[1]) ** 2 + (a[2] - b[2]) ** 2) ** 0.5


class G1Muscle(Muscle):
    """gym/walker.py:8-33: the G2 element with G1's default rest length."""
    distant = staticmethod(g1_distant)


class G1Skeleton(Skeleton):
    """gym/walker.py:49-55."""

    def __init__(self, p1: Point, p2: Point, x: float = None, k: float = 1000, dampk: float = 20):
        super().__init__(p1, p2, x=g1_distant(p1, p2) if x is None else x, k=k, dampk=dampk)


def _pts(xy, m=1):
    return [Phy(m, [0, 0, 0], [x, y, 0]) for x, y in xy]


def g1_leg2() -> Creature:
    """gym/walker.py:138-158 (marked "#fail" in the reference)."""
    p = _pts([(0, 100), (100, 100), (50, 50), (100, 0), (-100, 100), (-150, 50), (-100, 0)])
    sk = [G1Skeleton(p[a], p[b]) for a, b in ((0, 1), (0, 4), (1, 4), (1, 2), (2, 3), (4, 5), (5, 6))]
    m = [G1Muscle(p[a], p[b]) for a, b in ((1, 3), (4, 6), (0, 2), (0, 5))]
    return Creature(p, m, sk)


def g1_box() -> Creature:
    """gym/walker.py:160-171."""
    p = _pts([(-50, 0), (-50, 100), (50, 0), (50, 100)])
    sk = [G1Skeleton(p[0], p[1]), G1Skeleton(p[1], p[2]), G1Skeleton(p[2], p[3])]
    m = [G1Muscle(p[0], p[2]), G1Muscle(p[1], p[3])]
    return Creature(p, m, sk)


def g1_box2() -> Creature:
    """gym/walker.py:173-184."""
    p = _pts([(-50, 0), (-50, 100), (50, 100), (50, 0)])
    sk = [G1Skeleton(p[1], p[2])]
    m = [G1Muscle(p[a], p[b]) for a, b in ((0, 1), (0, 2), (3, 1), (3, 2))]
    return Creature(p, m, sk)


def g1_balance() -> Creature:
    """gym/walker.py:186-197."""
    p = _pts([(-50, 100), (50, 100), (0, 0), (0, 100)])
    sk = [G1Skeleton(p[0], p[1]), G1Skeleton(p[0], p[3]), G1Skeleton(p[1], p[3])]
    m = [G1Muscle(p[0], p[2]), G1Muscle(p[1], p[2])]
    return Creature(p, m, sk)


def g1_balance2() -> Creature:
    """gym/walker.py:199-210."""
    p = [Phy(5, [0, 0, 0], [-50, 100, 0]), Phy(5, [0, 0, 0], [50, 100, 0]), Phy(1, [0, 0, 0], [0, 0, 0]),
         Phy(0.1, [0, 0, 0], [0, 100, 0])]
    sk = [G1Skeleton(p[0], p[1]), G1Skeleton(p[0], p[3], k=10000), G1Skeleton(p[1], p[3], k=10000)]
    m = [G1Muscle(p[0], p[2]), G1Muscle(p[1], p[2])]
    return Creature(p, m, sk)


def g1_balance3() -> Creature:
    """gym/walker.py:212-223: the foot is a pinned DingPoint."""
    p = [Phy(1, [0, 0, 0], [-50, 100, 0]), Phy(1, [0, 0, 0], [50, 100, 0]), G1DingPoint(1, [0, 0, 0], [0, 0, 0]),
         Phy(0.1, [0, 0, 0], [0, 100, 0])]
    sk = [G1Skeleton(p[0], p[1]), G1Skeleton(p[0], p[3], k=20000), G1Skeleton(p[1], p[3], k=20000)]
    m = [G1Muscle(p[0], p[2]), G1Muscle(p[1], p[2])]
    return Creature(p, m, sk)


def g1_intrian() -> Creature:
    """gym/walker.py:225-234: three muscles, no skeleton."""
    p = _pts([(-50, 100), (50, 100), (0, 0)])
    m = [G1Muscle(p[0], p[2]), G1Muscle(p[1], p[2]), G1Muscle(p[0], p[1])]
    return Creature(p, m, [])


def g1_humanb() -> Creature:
    """gym/walker.py:236-253."""
    p = _pts([(25, 250), (-25, 200), (25, 150), (-25, 100), (25, 0), (-25, 0)])
    m = [G1Muscle(p[a], p[b]) for a, b in ((2, 4), (2, 5), (3, 4), (3, 5))]
    sk = [G1Skeleton(p[a], p[b]) for a, b in ((0, 1), (0, 2), (1, 2), (1, 3), (2, 3))]
    return Creature(p, m, sk)


def g1_insect() -> Creature:
    """gym/walker.py:255-293: 13 masses, 8 muscles, 15 skeletons."""
    p = _pts([(-75, 100), (-25, 100), (25, 100), (75, 100), (-100, 50), (-50, 50), (0, 50), (50, 50), (100, 50),
              (-75, 0), (-25, 0), (25, 0), (75, 0)])
    m = [G1Muscle(p[a], p[b]) for a, b in ((9, 4), (9, 5), (10, 5), (10, 6), (11, 6), (11, 7), (12, 7), (12, 8))]
    sk = [G1Skeleton(p[a], p[b]) for a, b in ((0, 1), (0, 4), (0, 5), (1, 2), (1, 5), (1, 6), (2, 3), (2, 6),
                                              (2, 7), (3, 7), (3, 8), (4, 5), (5, 6), (6, 7), (7, 8))]
    return Creature(p, m, sk)


def g1_box4() -> Creature:
    """gym/walker.py:295-312."""
    p = _pts([(-50, 100), (50, 100), (50, 0), (17, 0), (-17, 0), (-50, 0)])
    m = [G1Muscle(p[a], p[b]) for a, b in ((0, 2), (0, 3), (0, 4), (0, 5), (1, 2), (1, 3), (1, 4), (1, 5))]
    return Creature(p, m, [G1Skeleton(p[0], p[1])])


def g1_leg() -> Creature:
    """gym/walker.py:314-337."""
    p = _pts([(-50, 200), (50, 200), (-50, 140), (50, 140), (-50, 70), (50, 70), (-50, 0), (50, 0)])
    m = [G1Muscle(p[1], p[3]), G1Muscle(p[2], p[4]), G1Muscle(p[5], p[7])]
    sk = [G1Skeleton(p[a], p[b]) for a, b in ((0, 1), (0, 2), (1, 2), (2, 3), (3, 4), (3, 5), (4, 5), (4, 6),
                                              (5, 6), (6, 7))]
    return Creature(p, m, sk)


def g1_hat() -> Creature:
    """gym/walker.py:339-353."""
    p = _pts([(0, 150), (-50, 30), (50, 30), (-50, 0), (50, 0)])
    m = [G1Muscle(p[a], p[b]) for a, b in ((1, 3), (1, 4), (2, 3), (2, 4))]
    sk = [G1Skeleton(p[0], p[1]), G1Skeleton(p[0], p[2]), G1Skeleton(p[1], p[2])]
    return Creature(p, m, sk)


G1_BUILDERS: Dict[str, Callable[[], Creature]] = {
    "leg2": g1_leg2, "box": g1_box, "box2": g1_box2, "balance": g1_balance, "balance2": g1_balance2,
    "balance3": g1_balance3, "intrian": g1_intrian, "humanb": g1_humanb, "insect": g1_insect,
    "box4": g1_box4, "leg": g1_leg, "hat": g1_hat,
}


# ---------------------------------------------------------------------------------------------- G3
class G3Skeleton:
    """The builder API of gym/optimized_walker/walker.py:144-219 ``Skeleton(env)``: records points,
    springs and muscles in call order and turns them into a :class:`Creature`."""

    def __init__(self, env=None, spring_dampk: float = 20.0):
        self.env = env
        self.points: List[Point] = []
        self.springs: List[Skeleton] = []
        self.muscles: List[Muscle] = []
        self.spring_dampk = spring_dampk

    def add_point(self, m: float, pos, v=(0, 0, 0), r: float = None, color="black", is_ding: bool = False):
        """:157-177 (``is_ding`` -> a pinned DingPoint)."""
        pt = DingPoint(m, pos, v, r, color) if is_ding else Point(m, pos, v, r, color)
        self.points.append(pt)
        return pt

    def add_spring(self, point1, point2, k: float = 100, x: float = None, string: bool = False) -> None:
        """:179-191 -> env.add_spring (gym/optimized_walker/env.py:92-111, rest = norm in float32)."""
        self.springs.append(Skeleton(point1, point2, x=x, k=k, dampk=self.spring_dampk, string=string))

    def add_muscle(self, point1, point2, amp: float = 1.0, freq: float = 1.0, phase: float = 0.0,
                   power: float = 100.0, x: float = None) -> Muscle:
        """:193-209: an actuated spring of stiffness ``power`` and rest length ``x``."""
        mu = Muscle(point1, point2, x=x, k=power, dampk=self.spring_dampk)
        mu.amp, mu.freq, mu.phase, mu.power = amp, freq, phase, power
        self.muscles.append(mu)
        return mu

    def creature(self) -> Creature:
        return Creature(list(self.points), list(self.muscles), list(self.springs))


def g3_leg2(sk: G3Skeleton) -> Creature:
    """gym/optimized_walker/walker.py:377-414."""
    body = sk.add_point(5, (0, 10, 0), r=3)
    l1h, l1k, l1f = sk.add_point(1, (-5, 5, 0)), sk.add_point(1, (-5, -5, 0)), sk.add_point(2, (-5, -15, 0), r=2)
    l2h, l2k, l2f = sk.add_point(1, (5, 5, 0)), sk.add_point(1, (5, -5, 0)), sk.add_point(2, (5, -15, 0), r=2)
    sk.add_spring(body, l1h, k=500); sk.add_spring(l1h, l1k, k=300); sk.add_spring(l1k, l1f, k=300)
    sk.add_spring(body, l2h, k=500); sk.add_spring(l2h, l2k, k=300); sk.add_spring(l2k, l2f, k=300)
    sk.add_muscle(l1h, l1k, amp=0.1, freq=0.5, phase=0, power=200)
    sk.add_muscle(l1k, l1f, amp=0.1, freq=0.5, phase=0.5, power=200)
    sk.add_muscle(l2h, l2k, amp=0.1, freq=0.5, phase=0.5, power=200)
    sk.add_muscle(l2k, l2f, amp=0.1, freq=0.5, phase=0, power=200)
    return sk.creature()


def g3_box(sk: G3Skeleton, size: float = 10, mass: float = 1) -> Creature:
    """gym/optimized_walker/walker.py:417-451: a cube, 8 masses, 12 springs, no muscle."""
    h = size / 2
    p = [sk.add_point(mass, c) for c in ((-h, h, -h), (h, h, -h), (h, -h, -h), (-h, -h, -h),
                                         (-h, h, h), (h, h, h), (h, -h, h), (-h, -h, h))]
    for a, b in ((0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 6), (6, 7), (7, 4), (0, 4), (1, 5), (2, 6), (3, 7)):
        sk.add_spring(p[a], p[b], k=500)
    return sk.creature()


def _pendulum(sk: G3Skeleton, masses, ys) -> Creature:
    prev = sk.add_point(0, (0, 20, 0), is_ding=True, color="red")
    for m, y in zip(masses, ys):
        q = sk.add_point(m, (0, y, 0), **({"r": 3} if m == 5 else {"r": 2} if y == 0 else {}))
        sk.add_spring(prev, q, k=200)
        prev = q
    return sk.creature()


def g3_balance1(sk: G3Skeleton) -> Creature:
    """gym/optimized_walker/walker.py:454-471: pinned pivot (m = 0) and one bob."""
    return _pendulum(sk, [5], [0])


def g3_balance2(sk: G3Skeleton) -> Creature:
    """gym/optimized_walker/walker.py:474-493."""
    return _pendulum(sk, [2, 2], [10, 0])


def g3_balance3(sk: G3Skeleton) -> Creature:
    """gym/optimized_walker/walker.py:496-517."""
    return _pendulum(sk, [1.5, 1.5, 1.5], [15, 10, 0])


def g3_humanb(sk: G3Skeleton) -> Creature:
    """gym/optimized_walker/walker.py:520-584: 14 masses, 13 springs, 8 muscles."""
    head, torso = sk.add_point(3, (0, 30, 0), r=3, color="blue"), sk.add_point(10, (0, 20, 0), r=4)
    ls, le, lh = sk.add_point(2, (-8, 25, 0)), sk.add_point(1, (-15, 20, 0)), sk.add_point(1, (-20, 20, 0))
    rs, re, rh = sk.add_point(2, (8, 25, 0)), sk.add_point(1, (15, 20, 0)), sk.add_point(1, (20, 20, 0))
    lhip, lk, lf = sk.add_point(2, (-5, 10, 0)), sk.add_point(1, (-5, 0, 0)), sk.add_point(2, (-5, -10, 0), r=2)
    rhip, rk, rf = sk.add_point(2, (5, 10, 0)), sk.add_point(1, (5, 0, 0)), sk.add_point(2, (5, -10, 0), r=2)
    sk.add_spring(head, torso, k=500)
    sk.add_spring(torso, ls, k=400); sk.add_spring(ls, le, k=300); sk.add_spring(le, lh, k=200)
    sk.add_spring(torso, rs, k=400); sk.add_spring(rs, re, k=300); sk.add_spring(re, rh, k=200)
    sk.add_spring(torso, lhip, k=500); sk.add_spring(lhip, lk, k=400); sk.add_spring(lk, lf, k=400)
    sk.add_spring(torso, rhip, k=500); sk.add_spring(rhip, rk, k=400); sk.add_spring(rk, rf, k=400)
    sk.add_muscle(torso, le, amp=0.1, freq=0.3, phase=0, power=150)
    sk.add_muscle(ls, lh, amp=0.1, freq=0.3, phase=0.5, power=100)
    sk.add_muscle(torso, re, amp=0.1, freq=0.3, phase=0.5, power=150)
    sk.add_muscle(rs, rh, amp=0.1, freq=0.3, phase=0, power=100)
    sk.add_muscle(torso, lk, amp=0.1, freq=0.5, phase=0, power=200)
    sk.add_muscle(lhip, lf, amp=0.1, freq=0.5, phase=0.5, power=150)
    sk.add_muscle(torso, rk, amp=0.1, freq=0.5, phase=0.5, power=200)
    sk.add_muscle(rhip, rf, amp=0.1, freq=0.5, phase=0, power=150)
    return sk.creature()


def g3_insect(sk: G3Skeleton, legs: int = 6) -> Creature:
    """gym/optimized_walker/walker.py:587-639: legs // 2 body points, each with a 3-segment leg pair."""
    body_length = legs * 5
    nb = legs // 2
    body = []
    for i in range(nb):
        x = -body_length / 2 + i * (body_length / (nb - 1)) if legs > 2 else 0
        body.append(sk.add_point(2, (x, 5, 0), r=2))
    for i in range(len(body) - 1):
        sk.add_spring(body[i], body[i + 1], k=400)
    for i, bp in enumerate(body):
        bx = bp.pos[0]
        lu, ll = sk.add_point(1, (bx - 5, 0, 0)), sk.add_point(1, (bx - 10, -5, 0))
        lf = sk.add_point(1, (bx - 15, -10, 0), r=1.5)
        ru, rl = sk.add_point(1, (bx + 5, 0, 0)), sk.add_point(1, (bx + 10, -5, 0))
        rf = sk.add_point(1, (bx + 15, -10, 0), r=1.5)
        sk.add_spring(bp, lu, k=300); sk.add_spring(lu, ll, k=200); sk.add_spring(ll, lf, k=200)
        sk.add_spring(bp, ru, k=300); sk.add_spring(ru, rl, k=200); sk.add_spring(rl, rf, k=200)
        phase = i * (math.pi / nb)
        sk.add_muscle(bp, ll, amp=0.1, freq=0.8, phase=phase, power=100)
        sk.add_muscle(lu, lf, amp=0.1, freq=0.8, phase=phase + 0.5, power=80)
        sk.add_muscle(bp, rl, amp=0.1, freq=0.8, phase=phase + math.pi, power=100)
        sk.add_muscle(ru, rf, amp=0.1, freq=0.8, phase=phase + math.pi + 0.5, power=80)
    return sk.creature()


G3_BUILDERS: Dict[str, Callable[..., Creature]] = {
    "leg2": g3_leg2, "box": g3_box, "balance1": g3_balance1, "balance2": g3_balance2,
    "balance3": g3_balance3, "humanb": g3_humanb, "insect": g3_insect,
}


def build_creature(name: str, generation: int = 1, spring_dampk: float = 20.0, **kw) -> Creature:
    """One creature from the G1 (gym/walker.py), G2 (gym/optimized_walker.py) or G3
    (gym/optimized_walker/walker.py) builders."""
    if generation == 1:
        if name not in G1_BUILDERS:
            raise ValueError(f"unknown G1 topology {name!r}; have {sorted(G1_BUILDERS)}")
        return G1_BUILDERS[name]()
    if generation == 2:
        table = {"balance": create_balance_creature, "box": create_box_creature}
        if name not in table:
            raise ValueError(f"unknown G2 topology {name!r}; have {sorted(table)}")
        return table[name]()
    if generation == 3:
        if name not in G3_BUILDERS:
            raise ValueError(f"unknown G3 topology {name!r}; have {sorted(G3_BUILDERS)}")
        return G3_BUILDERS[name](G3Skeleton(spring_dampk=spring_dampk), **kw)
    raise ValueError("generation must be 1, 2 or 3")


def topology_spec(name: str, n: int = 1, generation: int = 1, **kw) -> dict:
    """``n`` copies of one builder's creature (a uniform batch)."""
    return replicate_spec(creatures_to_spec([build_creature(name, generation, **kw)]), n)


def mixed_spec(names_and_counts, generation: int = 1, **kw) -> dict:
    """A ragged batch: ``[(name, count), ...]`` creatures, in that order."""
    crs: List[Creature] = []
    for name, count in names_and_counts:
        crs.extend(build_creature(name, generation, **kw) for _ in range(int(count)))
    return creatures_to_spec(crs)


__all__ = ["Phy", "G1DingPoint", "g1_distant", "G1Muscle", "G1Skeleton", "G1_BUILDERS", "G3Skeleton",
           "G3_BUILDERS", "build_creature", "topology_spec", "mixed_spec"]
