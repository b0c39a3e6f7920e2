"""Reference-style CPU baseline — TEST / BENCH INFRASTRUCTURE ONLY (never the product path).

A per-object restatement of the reference's CPU loop, written the way gym/optimized_engine.py and
gym/optimized_walker.py run it: one Python object per mass holding float32 numpy 3-vectors, one object per
spring, and every force a ``Point.forced`` call on a tiny numpy array.  It exists to time the reference's
own execution model on the GPU box's host cores (SURVEY §8(d) "CPU baseline": the restated per-object loop of
gym/optimized_engine.py:259-311, single process and one process per core), next to the C port
(oracle/walker_oracle.c) and the GPU.  The step composes the engine primitives in the SURVEY §0.1 order with
the §8(c) fixes — the contract the C oracle and the kernel restate — so it also checks against the goldens
(tests/test_refstyle.py).

Only tests/ and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import os
import time

import numpy as np

f32 = np.float32
CONFIG_R = 1.6e-35          # Config.r, gym/engine.py:9


class RPoint:
    """gym/engine.py:24-59 (the fields the step touches)."""
    __slots__ = ("m", "pos", "v", "a", "old_a", "contact")

    def __init__(self, m, pos, v, old_a=None):
        self.m = float(m)
        self.pos = np.array(pos, dtype=f32)
        self.v = np.array(v, dtype=f32)
        self.a = np.zeros(3, dtype=f32)
        self.old_a = np.zeros(3, dtype=f32) if old_a is None else np.array(old_a, dtype=f32)
        self.contact = 0

    def zero(self):                                   # gym/engine.py:61-63
        self.a = np.zeros_like(self.v, dtype=f32)

    def forced(self, f):                              # gym/engine.py:65-67
        self.a += f / self.m

    def anti_forced(self, f_size, target):            # gym/engine.py:69-76
        direction = target.pos - self.pos
        distance = max(np.linalg.norm(direction).astype(float), CONFIG_R)
        self.forced(-f_size * direction / distance)


class RSpring:
    """One Muscle / Skeleton element: the engine spring (gym/engine.py:78-102, correct sign) then the
    relative-velocity damping of gym/optimized_walker.py:92-106."""
    __slots__ = ("p1", "p2", "x", "k", "c", "string", "x0", "lo", "hi", "stride")

    def __init__(self, p1, p2, x, k, c, string=False, minl=0.1, maxl=1.5, stride=2.0):
        self.p1, self.p2, self.x, self.k, self.c, self.string = p1, p2, f32(x), float(k), float(c), bool(string)
        self.x0, self.lo, self.hi, self.stride = self.x, float(minl), float(maxl), float(stride)

    def act(self, a):                                 # Muscle.act + regulation, gym/optimized_walker.py:27-35
        self.x += a
        self.x = max(self.x, self.x0 * self.lo)
        self.x = min(self.x, self.x0 * self.hi)

    def run(self):
        p1, p2 = self.p1, self.p2
        current = np.linalg.norm(p1.pos - p2.pos)
        dx = current - self.x
        f_size = 0 if (dx < 0 and self.string) else -dx * self.k
        p1.anti_forced(f_size, p2)
        p2.anti_forced(f_size, p1)
        direction = p2.pos - p1.pos
        if current > 0:
            direction = direction / current
        dk = np.dot(p1.v - p2.v, direction)
        damp_force = dk * self.c * direction
        p1.forced(-damp_force)
        p2.forced(damp_force)


class RWalker:
    """A Creature (gym/optimized_walker.py:108-172) inside its PhysicsEnv (gym/optimized_env.py:8-248)."""

    def __init__(self, spec, w, params):
        mo, eo = spec["mass_off"], spec["edge_off"]
        uo = np.concatenate([[0], np.cumsum(spec["n_muscles"])])
        acc = spec.get("acc")
        self.phys = [RPoint(spec["m"][q], spec["pos"][q], spec["vel"][q], None if acc is None else acc[q])
                     for q in range(mo[w], mo[w + 1])]
        A = int(spec["n_muscles"][w])
        self.springs = []
        for e in range(eo[w], eo[w + 1]):
            u = uo[w] + (e - eo[w])
            mus = e - eo[w] < A
            self.springs.append(RSpring(self.phys[spec["ei"][e]], self.phys[spec["ej"][e]], spec["rest"][e],
                                        spec["k"][e], spec["c"][e], bool(spec["flags"][e] & 1),
                                        *((spec["minl"][u], spec["maxl"][u], spec["stride"][u]) if mus else ())))
        self.muscles = self.springs[:A]
        self.p = params
        self.steps = 0

    def step(self, action, observe: bool = True):
        P = self.p
        for i in range(min(len(self.muscles), len(action))):      # Creature.act
            self.muscles[i].act(action[i])
        for p in self.phys:                                       # Creature.run: zero, then the springs
            p.zero()
        for s in self.springs:
            s.run()
        if P["pair_mode"] & 1:                                    # Point.gravity over the walker, gym/engine.py:128-137
            pts = self.phys
            for i in range(len(pts)):
                for j in range(i + 1, len(pts)):
                    r = np.linalg.norm(pts[i].pos - pts[j].pos).astype(float)
                    r = max(r, CONFIG_R)
                    f = -P["pair_g"] * pts[i].m * pts[j].m / (r ** 2)
                    pts[j].anti_forced(f, pts[i])
                    pts[i].anti_forced(f, pts[j])
        if P["pair_mode"] & 8 and len(self.phys) >= 2:           # G2 Point.gravity = gravity_vec,
            pts = self.phys                                       # gym/optimized_engine.py:167-193
            for p in pts:
                p.zero()
            for i in range(len(pts)):
                for j in range(i + 1, len(pts)):
                    p1, p2 = pts[i], pts[j]
                    direction = p2.pos - p1.pos
                    distance = np.linalg.norm(direction)
                    distance = max(distance, CONFIG_R)
                    f = -P["pair_g"] * p1.m * p2.m / (distance ** 2)
                    force = f * direction / distance
                    p1.forced(force)
                    p2.forced(-force)
        g, dampk, ground = P["g"], P["dampk"], P["ground"]
        for p in self.phys:                                       # gym/optimized_env.py:146-172
            p.forced(np.array([0, -g, 0], dtype=f32))
            p.forced(np.asarray(-dampk * p.v, dtype=f32))
            if p.pos[1] - ground < 0:
                p.contact = 1
                deep = p.pos[1] - ground
                p.forced(np.array([0, -P["groundk"] * deep, 0], dtype=f32))
                p.forced(np.array([0, -P["grounddamp"] * p.v[1], 0], dtype=f32))
                ff = np.abs(deep) * P["friction"]
                p.forced(np.array([-p.v[0] * ff, 0, -p.v[2] * ff], dtype=f32))
            else:
                p.contact = 0
        t = P["dt"]
        for p in self.phys:                                       # Point.run1, gym/engine.py:168-178
            p.v += p.a * t
            p.pos += p.v * t
            p.old_a = p.a.copy()
            p.zero()
        self.steps += 1
        return self.observe() if observe else None

    def observe(self):
        P = self.p
        d = 3 if P["in3d"] else 2
        mid = np.zeros(3, dtype=f32)                              # Creature.getstat, gym/optimized_walker.py:129
        for p in self.phys:
            mid += p.pos
        mid /= len(self.phys)
        s = []
        for p in self.phys:
            s.extend(((p.pos[:d] - mid[:d]) * P["pk"]).tolist())
            s.extend((p.v[:d] * P["vk"]).tolist())
            s.extend((p.old_a[:d] * P["ak"]).tolist())
        for mu in self.muscles:
            s.append(mu.x * P["mk"])
        obs = np.array(s)
        cy = np.mean([p.pos[1] for p in self.phys])               # _get_reward, gym/optimized_env.py:189-205
        vpen = -np.mean([np.linalg.norm(p.v) for p in self.phys]) * 0.1
        cpen = -sum(1 for p in self.phys if p.pos[1] - P["ground"] < 0) * 0.5
        reward = cy + vpen + cpen
        done = (self.steps >= P["max_steps"] or cy < P["ground"] - 50 or           # _is_done :207-230
                (all(np.linalg.norm(p.v) < 0.1 for p in self.phys) and self.steps > 100))
        ke = 0.5 * np.sum([p.m * np.linalg.norm(p.v) ** 2 for p in self.phys])     # _calculate_energy :240-248
        pe = np.sum([p.m * P["g"] * (p.pos[1] - P["ground"]) for p in self.phys])
        info = {"steps": self.steps, "centroid_position": np.mean([p.pos for p in self.phys], axis=0).tolist(),
                "total_energy": ke + pe}
        return obs, reward, done, info


DEFAULTS = dict(g=100.0, dampk=0.0, ground=0.0, groundk=1000.0, grounddamp=100.0, friction=100.0, dt=0.01,
                in3d=1, max_steps=1000, pk=1.0, vk=1.0, ak=1.0, mk=1.0, pair_mode=0, pair_g=9.8)


def walkers(spec, params=None):
    P = dict(DEFAULTS)
    P.update({k: v for k, v in (params or {}).items() if k in P})
    return [RWalker(spec, w, P) for w in range(len(spec["mass_off"]) - 1)]


def _timed(spec, params, actions, budget_s, observe=True):
    """Step every walker of spec with actions[t % T] until budget_s elapses; returns (walker-steps, seconds)."""
    ws = walkers(spec, params)
    n, t0 = 0, time.perf_counter()
    t = 0
    while True:
        a = actions[t % len(actions)]
        for w, wk in enumerate(ws):
            wk.step(a[w], observe)
        n += len(ws)
        t += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            return n, el


def _worker(args):
    return _timed(*args)


def throughput(spec, params, actions, budget_s: float, procs: int = 1, observe: bool = True) -> dict:
    """Env-steps/s of the per-object loop over `spec`: one process, or `procs` processes each stepping its own
    copy of the sample (one walker shard per core, spawned fresh: no GPU state is inherited).  observe=False
    times the physics alone (act, Creature.run, env forces, Point.run1), without getstat/reward/done/info."""
    if procs <= 1:
        n, el = _timed(spec, params, actions, budget_s, observe)
        return {"value": n / el, "procs": 1, "walker_steps": n, "seconds": el}
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        t0 = time.perf_counter()
        res = pool.map(_worker, [(spec, params, actions, budget_s, observe)] * procs)
        wall = time.perf_counter() - t0
    n = sum(r[0] for r in res)
    el = max(r[1] for r in res)
    return {"value": n / el, "procs": procs, "walker_steps": n, "seconds": el, "wall_incl_spawn": wall}


def host_cores() -> int:
    cores = len(os.sched_getaffinity(0))
    return max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
