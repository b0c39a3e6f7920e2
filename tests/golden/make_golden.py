#!/usr/bin/env python3
"""Generate golden step vectors by running the REFERENCE CPU engine (this container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--ref /root/reference]

What runs is the reference's own code, composed in the gym/env.py step order with the three
mechanical fixes SURVEY.md §8(c) lists (the reference's env loop cannot run as written):

  1. forces are passed to ``Point.forced`` as float32 ndarrays instead of lists
     (gym/env.py:32,39-41 and gym/optimized_env.py:148,162-172 raise TypeError at gym/engine.py:67);
  2. ``.pos`` is used for the G0 attribute ``.p`` (gym/env.py:35,38);
  3. ``c.run1()`` (gym/env.py:30, undefined) is replaced by the per-edge spring pass in edge order
     (muscles, then skeletons: gym/optimized_walker.py:124-127):
       spring   = reference ``gym.engine.Point.resilience`` (gym/engine.py:78-102, correct sign)
       damping  = reference ``gym/optimized_walker.py`` ``Skeleton.run`` executed with ``k=0`` so that
                  only its relative-velocity damping term acts (gym/optimized_walker.py:84-106; the
                  k=0 spring adds +/-0 to the accelerations, which is a no-op).
Everything else is the reference's code, called directly:
  * action          ``optimized_walker.Muscle.act/actdisp/regulation`` via ``Creature.act`` (:27-43,164-172)
  * integrator      ``gym.engine.Point.run1`` (gym/engine.py:168-178), or ``Point.run2`` (:180-190)
                    for the run2 scenario
  * pinned masses   ``optimized_engine.DingPoint`` objects (gym/optimized_engine.py:404-416: forced() is a
                    no-op), integrated by the same base ``Point.run1`` the envs call
  * observation     ``optimized_walker.Creature.getstat`` (:129-162)
  * reward/done/info ``optimized_env.PhysicsEnv._get_reward/_is_done/_get_info/_calculate_energy``
                    (gym/optimized_env.py:189-248), bound to a data shim
  * topologies      ``optimized_walker.create_balance_creature/create_box_creature`` (:176-224)
  * env forces      restated from gym/optimized_env.py:146-172 (the lines that raise as written),
                    each term one ``Point.forced`` call of the reference, in that order.
``state.pkl`` is read with ``walker_gym_amd.snapshot`` (an opcode walker that executes nothing),
never with ``pickle``.  Output: ``tests/golden/*.npz`` (inputs + per-step outputs; no pickles).
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys
import types
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from walker_gym_amd.snapshot import read_snapshot  # noqa: E402
from walker_gym_amd.synthetic import canonical_walkers, chain_walkers, ragged_walkers  # noqa: E402

f32 = np.float32


# --------------------------------------------------------------------------- reference import
def load_reference(ref: str):
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    for stub in ("turtle", "pygame"):
        sys.modules.setdefault(stub, types.ModuleType(stub))
    gymdir = os.path.join(ref, "gym")
    sys.path.insert(0, ref)
    sys.path.insert(0, gymdir)
    import gym.engine as E  # noqa: F401  (gym/engine.py, turtle stubbed)

    def by_path(name, fname):
        spec = importlib.util.spec_from_file_location(name, os.path.join(gymdir, fname))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        return mod

    by_path("optimized_engine", "optimized_engine.py")
    by_path("optimized_renderer", "optimized_renderer.py")
    OW = by_path("optimized_walker", "optimized_walker.py")      # the module, not the package
    OE = by_path("optimized_env", "optimized_env.py")
    return E, OW, OE


def load_g1_walker(ref: str, E):
    """gym/walker.py (G1) with the two names it uses but the reference no longer provides: ``Phy(m, v, p)``
    (undefined) and a DingPoint that is a real pinned point (gym/engine.py:569's never
    registers and has no ``pos``).  Both create reference engine objects; ``.p`` is the G0 attribute name
    gym/walker.py:5 reads, aliased to ``pos``."""
    spec = importlib.util.spec_from_file_location("walker_g1", os.path.join(ref, "gym", "walker.py"))
    G1 = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(G1)

    def Phy(m, v, p):
        pt = E.Point(m, p, v)
        pt.p = pt.pos
        return pt

    def Ding(m, v, p):
        pt = sys.modules["optimized_engine"].DingPoint(m, p, v)
        pt.p = pt.pos
        E.Point.points.append(pt)   # the env integrates it with the base Point.run1
        return pt

    G1.Phy, G1.DingPoint = Phy, Ding
    return G1


def load_g3(ref: str):
    """gym/optimized_walker/{core,env,walker}.py as a package without running its __init__ (renderer/demo
    imports; pygame is stubbed).  Returns (core, env, walker)."""
    d = os.path.join(ref, "gym", "optimized_walker")
    pkg = types.ModuleType("g3pkg")
    pkg.__path__ = [d]
    sys.modules["g3pkg"] = pkg
    mods = []
    for name in ("core", "renderer", "env", "walker"):
        spec = importlib.util.spec_from_file_location("g3pkg." + name, os.path.join(d, name + ".py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules["g3pkg." + name] = mod
        spec.loader.exec_module(mod)
        mods.append(mod)
    return mods[0], mods[2], mods[3]


# --------------------------------------------------------------------------- scenario plumbing
class Spec:
    """A batch in the flat CSR layout used by the oracle and the GPU path."""

    def __init__(self, m, pos, vel, mass_off, ei, ej, rest, k, c, flags, edge_off, n_muscles,
                 minl, maxl, stride, acc=None, pinned=None, mx=None, charge=None, radius=None, bounce_set=None):
        self.m = np.asarray(m, np.float32)
        # Point.bounce(k, other=<list>) per point: bit 0 calls bounce, bit 1 is in the list (None: every point, "*")
        self.bounce_set = None if bounce_set is None else np.asarray(bounce_set, np.uint8)
        self.charge = None if charge is None else np.asarray(charge, np.float64)   # Point.e
        self.radius = None if radius is None else np.asarray(radius, np.float64)   # Point.r
        self.pos = np.asarray(pos, np.float32).reshape(-1, 3)
        self.vel = np.asarray(vel, np.float32).reshape(-1, 3)
        self.acc = np.zeros_like(self.pos) if acc is None else np.asarray(acc, np.float32).reshape(-1, 3)
        self.mass_off = np.asarray(mass_off, np.int32)
        self.ei = np.asarray(ei, np.int32); self.ej = np.asarray(ej, np.int32)
        self.rest = np.asarray(rest, np.float32); self.k = np.asarray(k, np.float32)
        self.c = np.asarray(c, np.float32); self.flags = np.asarray(flags, np.uint8)
        self.edge_off = np.asarray(edge_off, np.int32)
        self.n_muscles = np.asarray(n_muscles, np.int32)
        self.minl = np.asarray(minl, np.float32); self.maxl = np.asarray(maxl, np.float32)
        self.stride = np.asarray(stride, np.float32)
        self.pinned = np.zeros(len(self.m), np.uint8) if pinned is None else np.asarray(pinned, np.uint8)

    @property
    def N(self):
        return len(self.mass_off) - 1

    def muscle_off(self):
        return np.concatenate([[0], np.cumsum(self.n_muscles)]).astype(np.int32)

    def arrays(self, prefix="in_"):
        d = {}
        for key in ("m", "pos", "vel", "acc", "mass_off", "ei", "ej", "rest", "k", "c", "flags",
                    "edge_off", "n_muscles", "minl", "maxl", "stride"):
            d[prefix + key] = getattr(self, key)
        for key in ("charge", "radius", "bounce_set"):
            if getattr(self, key) is not None:
                d[prefix + key] = getattr(self, key)
        if self.pinned.any():
            d[prefix + "pinned"] = self.pinned
        return d


def spec_from_creatures(creatures, point_index):
    """Pack reference Creature objects (with engine Points) into a Spec (topology + state)."""
    m, pos, vel, acc, mass_off, pinned = [], [], [], [], [0], []
    ei, ej, rest, k, c, flags, edge_off, nmus, minl, maxl, stride = [], [], [], [], [], [], [0], [], [], [], []
    ding = getattr(sys.modules.get("optimized_engine"), "DingPoint", ())
    for cr in creatures:
        base = len(m)
        for p in cr.phys:
            m.append(float(p.m)); pos.append(p.pos); vel.append(p.v); acc.append(p.old_a)
            pinned.append(1 if ding and isinstance(p, ding) else 0)
        mass_off.append(len(m))
        local = {id(p): q for q, p in enumerate(cr.phys)}
        for e in list(cr.muscles) + list(cr.skeletons):
            ei.append(local[id(e.p1)]); ej.append(local[id(e.p2)])
            rest.append(e.x); k.append(e.k); c.append(e.dampk); flags.append(getattr(e, "_string", 0))
        for mu in cr.muscles:
            minl.append(mu.minl); maxl.append(mu.maxl); stride.append(mu.stride)
        nmus.append(len(cr.muscles))
        edge_off.append(len(ei))
        del base
    return Spec(m, pos, vel, mass_off, ei, ej, rest, k, c, flags, edge_off, nmus, minl, maxl, stride, acc,
                pinned=pinned)


PARAM_KEYS = ("g", "dampk", "ground", "groundk", "grounddamp", "friction", "dt", "in3d", "max_steps",
              "pk", "vk", "ak", "mk", "midform", "conmid", "spring_mode", "integrator", "pair_mode", "pair_g",
              "pair_k", "pair_e", "bounce_k")
DEFAULT_PARAMS = dict(g=100.0, dampk=0.0, ground=0.0, groundk=1000.0, grounddamp=100.0, friction=100.0,
                      dt=0.01, in3d=1, max_steps=1000, pk=1.0, vk=1.0, ak=1.0, mk=1.0, midform=1,
                      conmid=0, spring_mode=0, integrator=1, pair_mode=0, pair_g=9.8,
                      pair_k=8.99e9, pair_e=16e-20, bounce_k=100.0)


class RefRun:
    """Drive the reference objects for one scenario and record every step."""

    def __init__(self, E, OW, OE, creatures, params, action_mode="cont", G1=None):
        self.E, self.OW, self.OE, self.G1 = E, OW, OE, G1
        self.cr = creatures
        self.p = dict(DEFAULT_PARAMS); self.p.update(params)
        self.action_mode = action_mode
        self.shims = []
        for cr in creatures:
            s = types.SimpleNamespace(creature=cr, ground=self.p["ground"], g=self.p["g"], steps=0,
                                      max_steps=int(self.p["max_steps"]), renderer=None)
            s._calculate_energy = (lambda s=s: OE.PhysicsEnv._calculate_energy(s))
            self.shims.append(s)

    def noise(self, noise):
        """PhysicsEnv.reset (gym/optimized_env.py:53-68) with host-supplied N(0, sigma) draws."""
        off = 0
        for cr in self.cr:
            for p in cr.phys:
                p.zero()
                p.v[0] += float(noise[off, 0])
                p.v[1] += float(noise[off, 1])
                if self.p["in3d"]:
                    p.v[2] += float(noise[off, 2])
                off += 1
        for s in self.shims:
            s.steps = 0

    def physics(self):
        E, OW, P = self.E, self.OW, self.p
        for cr in self.cr:
            for p in cr.phys:                      # Creature.run zero (gym/optimized_walker.py:120-121)
                p.zero()
            for e in list(cr.muscles) + list(cr.skeletons):
                if P["spring_mode"] == 1:          # G2-compat: the reference G2 element run as written
                    e.run()
                    continue
                e.p1.resilience(e.p2, e.x, e.k, bool(getattr(e, "_string", 0)))   # gym/engine.py:78
                OW.Skeleton(e.p1, e.p2, x=e.x, k=0, dampk=e.dampk).run()          # damping only
            if P["pair_mode"]:                     # gym/engine.py:114-147 over this walker's points only
                saved, g0, k0 = E.Point.points, E.Config.g, E.Config.k
                E.Point.points, E.Config.g, E.Config.k = list(cr.phys), P["pair_g"], P["pair_k"]
                if P["pair_mode"] & 1:
                    E.Point.gravity()              # :128-137
                if P["pair_mode"] & 2:
                    E.Point.coulomb()              # :139-147
                if P["pair_mode"] & 4:
                    bits = [getattr(p, "_golden_bounce", 3) for p in cr.phys]
                    if all(b == 3 for b in bits):
                        for p in cr.phys:          # :114-125, registry order, other = "*"
                            p.bounce(P["bounce_k"])
                    else:                          # the callers in registry order, each against one list
                        other = [p for p, b in zip(cr.phys, bits) if b & 2]
                        for p, b in zip(cr.phys, bits):
                            if b & 1:
                                p.bounce(P["bounce_k"], other=other)
                if P["pair_mode"] & 8:             # G2 Point.gravity = gravity_vec (gym/optimized_engine.py:167-197)
                    OEng = sys.modules["optimized_engine"]
                    saved2, og = OEng.Point.points, OEng.Config.g
                    OEng.Point.points, OEng.Config.g = list(cr.phys), P["pair_g"]
                    OEng.Point.gravity_vec()
                    OEng.Point.points, OEng.Config.g = saved2, og
                if P["pair_mode"] & 16:
                    for p in cr.phys:              # gym/engine.py:150-158, every point in registry order
                        p.electrostatic()
                E.Point.points, E.Config.g, E.Config.k = saved, g0, k0
            for p in cr.phys:                      # gym/optimized_env.py:146-172 with forces as f32 arrays
                p.forced(np.array([0, -P["g"], 0], dtype=f32))
                p.forced(np.asarray(-P["dampk"] * p.v, dtype=f32))
                if p.pos[1] - P["ground"] < 0:
                    p.color = "red"; p.r = 3
                    deep = p.pos[1] - P["ground"]
                    p.forced(np.array([0, -P["groundk"] * deep, 0], dtype=f32))
                    p.forced(np.array([0, -P["grounddamp"] * p.v[1], 0], dtype=f32))
                    friction_force = np.abs(deep) * P["friction"]
                    p.forced(np.array([-p.v[0] * friction_force, 0, -p.v[2] * friction_force], dtype=f32))
                else:
                    p.color = "black"; p.r = 1
        if P["integrator"] == 2:
            E.Point.run2(P["dt"])                  # gym/engine.py:180-190
        else:
            E.Point.run1(P["dt"])                  # gym/engine.py:168-178

    def act(self, actions):
        for w, cr in enumerate(self.cr):
            a = actions[w]
            if self.action_mode == "disc":
                cr.actdisp([bool(x) for x in a])
            else:
                cr.act(a)

    def observe(self):
        P = self.p
        out = []
        for s in self.shims:
            if P["midform"] == 2:   # G1 Creature.getstat (gym/walker.py:83-101: mid is the SUM of positions)
                obs = np.array(self.G1.Creature.getstat(s.creature, bool(P["in3d"]), P["pk"], P["vk"], P["ak"],
                                                        P["mk"], True, bool(P["conmid"])))
            else:
                obs = np.array(self.OW.Creature.getstat(s.creature, bool(P["in3d"]), P["pk"], P["vk"], P["ak"],
                                                        P["mk"], bool(P["midform"]), bool(P["conmid"])))
            o32 = obs.astype(f32)
            assert np.array_equal(o32.astype(np.float64), obs, equal_nan=True), "obs not f32-exact"
            out.append(o32)
        return out

    def rewards(self):
        OE = self.OE
        r, d, cen, en, st = [], [], [], [], []
        for s in self.shims:
            r.append(OE.PhysicsEnv._get_reward(s))
            d.append(OE.PhysicsEnv._is_done(s))
            info = OE.PhysicsEnv._get_info(s)
            cen.append(info["centroid_position"]); en.append(info["total_energy"]); st.append(info["steps"])
        return (np.array(r, f32), np.array(d, np.uint8), np.array(cen, f32), np.array(en, f32),
                np.array(st, np.int32))

    def step(self, actions):
        if actions is not None:
            self.act(actions)
        self.physics()
        for s in self.shims:
            s.steps += 1


def record(run: RefRun, spec_fn, T, actions, noise=None, momentum=False):
    """Run T steps; returns dict of stacked per-step outputs (plus reset observation).  momentum: also record each
    walker's Point.momentum() (gym/engine.py:160-166) over its own points after every step (out_momentum)."""
    rec = {k: [] for k in ("pos", "vel", "acc", "mx", "contact", "obs", "reward", "done", "centroid",
                           "energy", "steps")}
    if momentum:
        rec["momentum"] = []
    if noise is not None:
        run.noise(noise)
    obs0 = run.observe()
    for t in range(T):
        run.step(None if actions is None else actions[t])
        pos, vel, acc, mx, con = [], [], [], [], []
        for cr in run.cr:
            for p in cr.phys:
                pos.append(p.pos.copy()); vel.append(p.v.copy()); acc.append(np.asarray(p.old_a).copy())
                con.append(1 if p.color == "red" else 0)
            for mu in cr.muscles:
                mx.append(np.float32(mu.x))
        obs = run.observe()
        r, d, cen, en, st = run.rewards()
        rec["pos"].append(np.array(pos, f32)); rec["vel"].append(np.array(vel, f32))
        rec["acc"].append(np.array(acc, f32)); rec["mx"].append(np.array(mx, f32).reshape(-1))
        rec["contact"].append(np.array(con, np.uint8))
        rec["obs"].append(pad_obs(obs)); rec["reward"].append(r); rec["done"].append(d)
        rec["centroid"].append(cen); rec["energy"].append(en); rec["steps"].append(st)
        if momentum:
            E, mom = run.E, []
            saved = E.Point.points
            for cr in run.cr:
                E.Point.points = list(cr.phys)
                with np.errstate(all="ignore"):   # a diverged walker's momentum is inf / NaN, as the reference's
                    mom.append(np.asarray(E.Point.momentum(), f32))
            E.Point.points = saved
            rec["momentum"].append(np.array(mom, f32))
    out = {"out_" + k: np.stack(v) for k, v in rec.items()}
    out["out_obs0"] = pad_obs(obs0)
    out["out_obs_len"] = np.array([len(o) for o in obs0], np.int32)
    return out


def pad_obs(obs_list):
    D = max(len(o) for o in obs_list)
    out = np.zeros((len(obs_list), D), f32)
    for w, o in enumerate(obs_list):
        out[w, :len(o)] = o
    return out


def params_array(p):
    # integrator is recorded only where it is not the default, so the older fixtures stay byte-stable
    keep = lambda k: (k != "integrator" or p[k] != 1) and (k not in ("pair_mode", "pair_g") or p["pair_mode"] != 0) and \
        (k not in ("pair_k", "pair_e", "bounce_k") or p["pair_mode"] > 1)
    return {"param_" + k: np.array(p[k]) for k in PARAM_KEYS if keep(k)}


# --------------------------------------------------------------------------- creature builders
def creatures_from_spec(E, OW, spec: Spec):
    """Instantiate reference engine Points + reference Muscle/Skeleton objects for a Spec."""
    crs = []
    mo = spec.muscle_off()
    for w in range(spec.N):
        a, b = spec.mass_off[w], spec.mass_off[w + 1]
        phys = []
        for q in range(a, b):
            if spec.pinned[q]:
                # the reference's DingPoint(m, p, v) (gym/optimized_engine.py:404-410), run by E.Point.run1
                p = sys.modules["optimized_engine"].DingPoint(float(spec.m[q]), spec.pos[q].copy(), spec.vel[q].copy())
                E.Point.points.append(p)
            else:
                p = E.Point(float(spec.m[q]), spec.pos[q].copy(), spec.vel[q].copy())
            if spec.charge is not None:
                p.e = float(spec.charge[q])
            if spec.radius is not None:
                p.r = float(spec.radius[q])
            if spec.bounce_set is not None:
                p._golden_bounce = int(spec.bounce_set[q])   # (read by RefRun.physics, not by the reference)
            phys.append(p)
        for q, p in zip(range(a, b), phys):
            p.old_a = spec.acc[q].copy()
        e0, e1 = spec.edge_off[w], spec.edge_off[w + 1]
        A = int(spec.n_muscles[w])
        mus, sks = [], []
        for e in range(e0, e1):
            p1, p2 = phys[spec.ei[e]], phys[spec.ej[e]]
            if e - e0 < A:
                u = mo[w] + (e - e0)
                el = OW.Muscle(p1, p2, x=np.float32(spec.rest[e]), k=float(spec.k[e]),
                               maxl=float(spec.maxl[u]), minl=float(spec.minl[u]),
                               stride=float(spec.stride[u]), dampk=float(spec.c[e]))
                mus.append(el)
            else:
                el = OW.Skeleton(p1, p2, x=np.float32(spec.rest[e]), k=float(spec.k[e]), dampk=float(spec.c[e]))
                sks.append(el)
            el._string = int(spec.flags[e] & 1)
        crs.append(OW.Creature(phys, mus, sks))
    return crs


def reference_builders(E, OW, which, n=1):
    """Use the reference's own create_*_creature with engine Points (patching its Point name)."""
    OW.Point = E.Point
    f = {"balance": OW.create_balance_creature, "box": OW.create_box_creature}[which]
    crs = [f() for _ in range(n)]
    for cr in crs:
        for e in list(cr.muscles) + list(cr.skeletons):
            e._string = 0
    return crs


# --------------------------------------------------------------------------- scenarios
# Each fixture draws from its own generator, seeded by its name (scenario_rng): adding, removing or reordering
# scenarios never changes another fixture, and `--only NAME` regenerates NAME alone (tests/test_golden_regen.py
# does that for one cheap fixture of each script and compares the arrays with the committed file).
def scenario_rng(name: str) -> np.random.Generator:
    return np.random.default_rng(zlib.crc32(name.encode()))


SCENARIOS = []


def scenario(*names):
    """Register a scenario function writing the fixtures `names`."""
    def deco(fn):
        SCENARIOS.append((names, fn))
        return fn
    return deco


class Ctx:
    def __init__(self, E, OW, OE, args):
        self.E, self.OW, self.OE, self.args = E, OW, OE, args
        self.written = []

    def fresh(self):
        self.E.Point.points = []
        self.E.Point.r_points = {}

    def save(self, name, run, spec, T, actions, noise=None, extra=None, action_mode="cont", momentum=False):
        outs = record(run, None, T, actions, noise, momentum)
        blob = {}
        blob.update(spec.arrays())
        blob.update(params_array(run.p))
        blob["actions"] = (np.zeros((T, spec.N, 0), f32) if actions is None
                           else np.asarray(actions, f32))
        blob["action_mode"] = np.array(0 if action_mode == "cont" else 1, np.int32)
        blob["noise"] = np.zeros((0, 3), f32) if noise is None else np.asarray(noise, f32)
        blob["numpy_version"] = np.array(np.__version__)
        blob.update(outs)
        if extra:
            blob.update(extra)
        self.write(name, blob)

    def write(self, name, blob, sub=None):
        d = os.path.join(self.args.out, sub) if sub else self.args.out
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, name + ".npz")
        np.savez_compressed(path, **blob)
        self.written.append((name, os.path.getsize(path)))


@scenario("state_pkl")
def sc_state_pkl(c):
    """A. state.pkl (2 masses, no springs), 100 steps, no noise: SURVEY §0.1 known-answer case."""
    E, OW, OE = c.E, c.OW, c.OE
    c.fresh()
    pts, _ = read_snapshot(os.path.join(c.args.ref, "state.pkl"))
    phys = []
    for sp in pts:
        p = E.Point(sp.m, sp.pos.copy(), sp.v.copy())
        p.a = sp.a.copy(); p.old_a = sp.old_a.copy()
        phys.append(p)
    cr = OW.Creature(phys, [], [])
    spec = spec_from_creatures([cr], None)
    c.save("state_pkl", RefRun(E, OW, OE, [cr], dict(in3d=1)), spec, 100, None)


@scenario("balance_2d", "balance_3d")
def sc_balance(c):
    """B. Balance-v0 (reference builder), 2D and 3D observation, U(-1,1) actions, 100 steps."""
    for in3d in (0, 1):
        name = f"balance_{'3d' if in3d else '2d'}"
        c.fresh()
        crs = reference_builders(c.E, c.OW, "balance", 2)
        spec = spec_from_creatures(crs, None)
        acts = scenario_rng(name).uniform(-1, 1, (100, 2, 2)).astype(f32)
        c.save(name, RefRun(c.E, c.OW, c.OE, crs, dict(in3d=in3d)), spec, 100, acts)


@scenario("box_3d")
def sc_box(c):
    """C. Box-v0, 3D, larger actions (hits the muscle clamps), 100 steps."""
    c.fresh()
    crs = reference_builders(c.E, c.OW, "box", 2)
    spec = spec_from_creatures(crs, None)
    acts = scenario_rng("box_3d").uniform(-20, 20, (100, 2, 4)).astype(f32)
    c.save("box_3d", RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1)), spec, 100, acts)


@scenario("info_extras")
def sc_info_extras(c):
    """Opt-in info (ABI 10): a mixed batch — two Box-v0 walkers whose state goes non-finite at step 37 (as in box_3d)
    beside two Balance-v0 walkers — 60 steps, with every walker's Point.momentum() (gym/engine.py:160-166) over its
    own points after each step (out_momentum); the non-finite flag is read off out_pos / out_vel / out_acc."""
    c.fresh()
    crs = reference_builders(c.E, c.OW, "box", 2) + reference_builders(c.E, c.OW, "balance", 2)
    spec = spec_from_creatures(crs, None)
    rng = scenario_rng("info_extras")
    acts = np.zeros((60, 4, 4), f32)
    acts[:, :2] = rng.uniform(-20, 20, (60, 2, 4))
    acts[:, 2:, :2] = rng.uniform(-1, 1, (60, 2, 2))
    c.save("info_extras", RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1)), spec, 60, acts, momentum=True)


@scenario("canonical")
def sc_canonical(c):
    """D. canonical synthetic walker (M=16, K=40, A=8), 4 walkers, U(-1,1) actions, 100 steps."""
    c.fresh()
    spec = Spec(**canonical_walkers(4, seed=7))
    crs = creatures_from_spec(c.E, c.OW, spec)
    acts = scenario_rng("canonical").uniform(-1, 1, (100, 4, 8)).astype(f32)
    c.save("canonical", RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1)), spec, 100, acts)


@scenario("random_1step")
def sc_random_1step(c):
    """E. 1-step transitions from 1,000 random states (contact and no contact, random velocities)."""
    rng = scenario_rng("random_1step")
    c.fresh()
    base = canonical_walkers(1000, seed=11)
    base["pos"] = base["pos"] + rng.normal(0, 3, base["pos"].shape).astype(f32)
    base["pos"][:, 1] -= rng.uniform(0, 12, len(base["pos"])).astype(f32)     # many below ground
    base["vel"] = rng.normal(0, 20, base["vel"].shape).astype(f32)
    base["acc"] = rng.normal(0, 5, base["vel"].shape).astype(f32)
    spec = Spec(**base)
    crs = creatures_from_spec(c.E, c.OW, spec)
    acts = rng.uniform(-1, 1, (1, 1000, 8)).astype(f32)
    c.save("random_1step", RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1)), spec, 1, acts)


@scenario("ragged")
def sc_ragged(c):
    """F. ragged mixed-topology batch, string edges, non-default env params, 50 steps."""
    c.fresh()
    spec = Spec(**ragged_walkers(12, seed=5, string_frac=0.15))
    crs = creatures_from_spec(c.E, c.OW, spec)
    Amax = int(spec.n_muscles.max())
    acts = scenario_rng("ragged").uniform(-2, 2, (50, spec.N, Amax)).astype(f32)
    run = RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1, g=60.0, dampk=0.5, ground=-3.0, groundk=800.0,
                                            grounddamp=50.0, friction=30.0, dt=0.005))
    c.save("ragged", run, spec, 50, acts)


@scenario("reset_noise")
def sc_reset_noise(c):
    """G. reset noise (host-injected N(0,0.1) draws, as PhysicsEnv.reset adds them) + 20 steps."""
    rng = scenario_rng("reset_noise")
    c.fresh()
    crs = reference_builders(c.E, c.OW, "balance", 3)
    spec = spec_from_creatures(crs, None)
    noise = rng.normal(0, 0.1, (spec.mass_off[-1], 3)).astype(f32)
    acts = rng.uniform(-1, 1, (20, 3, 2)).astype(f32)
    c.save("reset_noise", RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1)), spec, 20, acts, noise=noise)


@scenario("obs_variants")
def sc_obs_variants(c):
    """H. observation variants: scales, midform off, conmid on, 2D; partial actions (len(a) < A)."""
    c.fresh()
    spec = Spec(**canonical_walkers(3, seed=3))
    crs = creatures_from_spec(c.E, c.OW, spec)
    acts = scenario_rng("obs_variants").uniform(-1, 1, (10, 3, 5)).astype(f32)   # 5 of 8 muscles act
    run = RefRun(c.E, c.OW, c.OE, crs, dict(in3d=0, pk=0.5, vk=2.0, ak=0.25, mk=3.0, midform=0, conmid=1))
    c.save("obs_variants", run, spec, 10, acts)


@scenario("edge_cases")
def sc_edge_cases(c):
    """I. edge cases: coincident masses (zero-length edge), compressed strings, discrete actions."""
    c.fresh()
    sp = canonical_walkers(2, seed=9)
    sp["pos"][1] = sp["pos"][0]                                     # masses 0,1 coincide in walker 0
    e0 = int(sp["edge_off"][0])
    sp["ei"][e0 + 30], sp["ej"][e0 + 30] = 0, 1                     # skeleton edge between them
    sp["rest"][e0 + 30] = 0.0
    sp["flags"][e0 + 31:e0 + 40] = 1                                # strings
    sp["rest"][e0 + 31:e0 + 40] *= 1.3                              # slack strings (compressed)
    spec = Spec(**sp)
    crs = creatures_from_spec(c.E, c.OW, spec)
    acts = (scenario_rng("edge_cases").uniform(0, 1, (30, 2, 8)) > 0.5).astype(f32)
    run = RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1), action_mode="disc")
    c.save("edge_cases", run, spec, 30, acts, action_mode="disc")


@scenario("g2_compat")
def sc_g2_compat(c):
    """J. G2-compat: the reference's optimized_walker Muscle/Skeleton.run as written (inverted sign)."""
    c.fresh()
    crs = reference_builders(c.E, c.OW, "balance", 1)
    spec = spec_from_creatures(crs, None)
    acts = scenario_rng("g2_compat").uniform(-1, 1, (60, 1, 2)).astype(f32)
    c.save("g2_compat", RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1, spring_mode=1)), spec, 60, acts)


@scenario("pinned_balance3", "pinned_canonical")
def sc_pinned(c):
    """K. pinned masses (DingPoint): the G1 balance3 topology (gym/walker.py:212-223, Phy(m, v, p) argument order as
    its DingPoint(m, v, p) at gym/engine.py:570) and canonical walkers with two pinned masses each; reset noise
    moves the pinned masses (a stays 0), 60 steps."""
    b3 = dict(m=[1, 1, 1, 0.1], pos=[[-50, 100, 0], [50, 100, 0], [0, 0, 0], [0, 100, 0]], vel=np.zeros((4, 3)),
              mass_off=[0, 4], ei=[0, 1, 0, 0, 1], ej=[2, 2, 1, 3, 3], k=[1000, 1000, 1000, 20000, 20000],
              c=[20] * 5, flags=[0] * 5, edge_off=[0, 5], n_muscles=[2], minl=[0.1, 0.1], maxl=[1.5, 1.5],
              stride=[2, 2], pinned=[0, 0, 1, 0])
    b3["rest"] = [float(np.linalg.norm(np.asarray(b3["pos"][i], f32) - np.asarray(b3["pos"][j], f32)))
                  for i, j in zip(b3["ei"], b3["ej"])]
    cw = canonical_walkers(3, seed=21)
    cw["pinned"] = np.zeros(48, np.uint8); cw["pinned"][[0, 5, 16 + 3, 16 + 12, 32 + 15, 32 + 7]] = 1
    for name, sp, in3d, A in (("pinned_balance3", b3, 0, 2), ("pinned_canonical", cw, 1, 8)):
        rng = scenario_rng(name)
        c.fresh()
        spec = Spec(**sp)
        crs = creatures_from_spec(c.E, c.OW, spec)
        noise = rng.normal(0, 0.5, (spec.mass_off[-1], 3)).astype(f32)
        acts = rng.uniform(-1, 1, (60, spec.N, A)).astype(f32)
        c.save(name, RefRun(c.E, c.OW, c.OE, crs, dict(in3d=in3d)), spec, 60, acts, noise=noise)


@scenario("run2_canonical", "run2_balance")
def sc_run2(c):
    """L. Point.run2 integrator (gym/engine.py:180-190) on canonical walkers and Balance-v0, 60 steps."""
    c.fresh()
    spec = Spec(**canonical_walkers(3, seed=23))
    crs = creatures_from_spec(c.E, c.OW, spec)
    acts = scenario_rng("run2_canonical").uniform(-1, 1, (60, 3, 8)).astype(f32)
    c.save("run2_canonical", RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1, integrator=2)), spec, 60, acts)
    c.fresh()
    crs = reference_builders(c.E, c.OW, "balance", 2)
    spec = spec_from_creatures(crs, None)
    acts = scenario_rng("run2_balance").uniform(-1, 1, (60, 2, 2)).astype(f32)
    c.save("run2_balance", RefRun(c.E, c.OW, c.OE, crs, dict(in3d=0, integrator=2)), spec, 60, acts)


def _balance_spec(c, charge=None, radius=None):
    """Two reference Balance-v0 creatures as a Spec (the builder's own points), with optional charges / radii."""
    c.fresh()
    base = spec_from_creatures(reference_builders(c.E, c.OW, "balance", 2), None)
    c.fresh()
    return Spec(**{k: getattr(base, k) for k in ("m", "pos", "vel", "mass_off", "ei", "ej", "rest", "k", "c",
                                                 "flags", "edge_off", "n_muscles", "minl", "maxl", "stride",
                                                 "acc", "pinned")}, charge=charge, radius=radius)


def _shrunk(seed):
    """The canonical lattice shrunk to spacing 4 so that neighbours collide (Point.bounce)."""
    sp = canonical_walkers(3, seed=seed)
    sp["pos"] = (sp["pos"] * np.float32(0.4)).astype(f32)
    sp["rest"] = (sp["rest"] * np.float32(0.4)).astype(f32)
    return sp


@scenario("pair_gravity_canonical", "pair_gravity_balance", "pair_coulomb_canonical", "pair_bounce_canonical",
          "pair_all_balance", "pair_electrostatic_canonical", "pair_g2_gravity_canonical", "pair_all_bits_balance")
def sc_pairs(c):
    """O/P. per-walker pair passes after the springs, in bit order (gym/engine.py:114-158 and
    gym/optimized_engine.py:167-197 restricted to each walker's points): 1 Point.gravity, 2 Point.coulomb, 4
    Point.bounce, 8 G2 Point.gravity (gravity_vec: every a zeroed first, float32 pairs), 16 Point.electrostatic of
    every point.  Config.g / Config.k raised so the forces matter; charges U(-3, 3); bounce on the shrunk lattice
    with initial radii U(1.5, 3) (after the first env pass the radii are the env's 3 / 1,
    gym/optimized_env.py:156,175); 60 steps."""
    cases = (("pair_gravity_canonical", lambda r: Spec(**canonical_walkers(3, seed=31)), 1, 8, 1, dict(pair_g=2000.0)),
             ("pair_gravity_balance", lambda r: _balance_spec(c), 0, 2, 1, dict(pair_g=5.0e4)),
             ("pair_coulomb_canonical", lambda r: Spec(**canonical_walkers(3, seed=41), charge=r.uniform(-3, 3, 48)),
              1, 8, 2, dict(pair_k=1.0e4)),
             ("pair_bounce_canonical", lambda r: Spec(**_shrunk(43), radius=r.uniform(1.5, 3.0, 48)), 1, 8, 4,
              dict(bounce_k=2000.0)),
             ("pair_all_balance", lambda r: _balance_spec(c, charge=r.uniform(-2, 2, 8)), 0, 2, 7,
              dict(pair_g=5.0e4, pair_k=2.0e5, bounce_k=500.0)),
             ("pair_electrostatic_canonical",
              lambda r: Spec(**canonical_walkers(3, seed=47), charge=r.uniform(-3, 3, 48)), 1, 8, 16,
              dict(pair_k=1.0e4)),
             ("pair_g2_gravity_canonical", lambda r: Spec(**canonical_walkers(3, seed=53)), 1, 8, 8,
              dict(pair_g=2000.0)),
             ("pair_all_bits_balance", lambda r: _balance_spec(c, charge=r.uniform(-2, 2, 8)), 0, 2, 31,
              dict(pair_g=5.0e4, pair_k=2.0e5, bounce_k=500.0)))
    for name, mk, in3d, A, pm, extra_p in cases:
        rng = scenario_rng(name)
        c.fresh()
        spec = mk(rng)
        crs = creatures_from_spec(c.E, c.OW, spec)
        acts = rng.uniform(-1, 1, (60, spec.N, A)).astype(f32)
        c.save(name, RefRun(c.E, c.OW, c.OE, crs, dict(in3d=in3d, pair_mode=pm, **extra_p)), spec, 60, acts)


@scenario("pair_bounce_subset_canonical", "pair_bounce_subset_lattice25")
def sc_bounce_subset(c):
    """O2. Point.bounce(k, other=<list>) (gym/engine.py:114-125) with a proper subset: on each walker the points with
    bit 0 call p.bounce(k, other=L) in registry order, L = the points with bit 1 in registry order (bits U{0..3} per
    point, so callers outside L, L members that never call, and both); the shrunk canonical lattice (lean kernel) and a
    shrunk 25-mass lattice (workgroup kernel), radii U(1.5, 3), 60 steps."""
    def shrunk25(seed):
        sp = canonical_walkers(3, seed=seed, M=25, K=60, A=10)
        sp["pos"] = (sp["pos"] * np.float32(0.4)).astype(f32)
        sp["rest"] = (sp["rest"] * np.float32(0.4)).astype(f32)
        return sp
    cases = (("pair_bounce_subset_canonical", lambda r: Spec(**_shrunk(59), radius=r.uniform(1.5, 3.0, 48),
                                                            bounce_set=r.integers(0, 4, 48)), 8),
             ("pair_bounce_subset_lattice25", lambda r: Spec(**shrunk25(61), radius=r.uniform(1.5, 3.0, 75),
                                                            bounce_set=r.integers(0, 4, 75)), 10))
    for name, mk, A in cases:
        rng = scenario_rng(name)
        c.fresh()
        spec = mk(rng)
        crs = creatures_from_spec(c.E, c.OW, spec)
        acts = rng.uniform(-1, 1, (60, spec.N, A)).astype(f32)
        c.save(name, RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1, pair_mode=4, bounce_k=2000.0)), spec, 60, acts)


@scenario(*[f"chain_engine_gravity_{n}" for n in (10, 50, 100, 200)])
def sc_chain_engine_gravity(c):
    """performance_demo's chain topology (gym/performance_demo.py:30-44: U(-100,100) positions, U(-10,10) velocities,
    Skeleton(k=50) links) with gym/ENGINE.py's Point.gravity (:128-137, the float64 anti_forced path) over the
    walker's points after its springs, no env gravity (g = 0) and no ground; one walker each, 40 steps.  (The loop
    performance_demo itself runs uses optimized_engine's Point.gravity = gravity_vec: perfdemo_chain_* below.)"""
    for n_pts in (10, 50, 100, 200):
        c.fresh()
        spec = Spec(**chain_walkers(1, n_pts, seed=n_pts))
        crs = creatures_from_spec(c.E, c.OW, spec)
        run = RefRun(c.E, c.OW, c.OE, crs, dict(in3d=1, g=0.0, ground=-1.0e6, pair_mode=1, pair_g=9.8))
        c.save(f"chain_engine_gravity_{n_pts}", run, spec, 40, None)


class PerfDemoRun(RefRun):
    """gym/performance_demo.py:52-58 as written, one step: creature.run(); Point.gravity(); Point.run1(0.01), with
    the G2 modules it imports (optimized_engine.Point, optimized_walker.Creature/Skeleton; the G2 module, loaded by
    path: the package shadows it).  Point.gravity is gravity_vec (gym/optimized_engine.py:167-197), which
    zeroes every a first.  Observation / reward / info are the same env shims as every other fixture (g = 0, ground
    far below), so the fixture also pins the outputs of the step the GPU runs for it."""

    def __init__(self, OEng, *a, **k):
        super().__init__(*a, **k)
        self.OEng = OEng

    def physics(self):
        for cr in self.cr:
            cr.run()                      # gym/optimized_walker.py:117-127 (G2 elements; discarded by gravity_vec)
        self.OEng.Point.gravity()         # gym/optimized_engine.py:195-197 -> gravity_vec
        self.OEng.Point.run1(self.p["dt"])   # gym/optimized_engine.py:258-272


@scenario(*[f"perfdemo_chain_{n}" for n in (10, 50, 100, 200)])
def sc_perfdemo(c):
    """The performance_demo loop as written (PerfDemoRun) for N in {10, 50, 100, 200}: chain_walkers' topology and
    initial state in G2 Points (m = 1 as Point(1, pos, v)), G2 Skeleton(k=50) links, 40 steps of dt = 0.01."""
    OEng = sys.modules["optimized_engine"]
    for n_pts in (10, 50, 100, 200):
        OEng.Point.clear()
        spec = Spec(**chain_walkers(1, n_pts, seed=1000 + n_pts))
        pts = [OEng.Point(1, spec.pos[q].copy(), spec.vel[q].copy(), color="blue") for q in range(n_pts)]
        sks = [c.OW.Skeleton(pts[i], pts[i + 1], x=np.float32(spec.rest[i]), k=float(spec.k[i]),
                             dampk=float(spec.c[i])) for i in range(n_pts - 1)]
        for e in sks:
            e._string = 0
        cr = c.OW.Creature(pts, [], sks)
        run = PerfDemoRun(OEng, c.E, c.OW, c.OE, [cr], dict(in3d=1, g=0.0, ground=-1.0e6, pair_mode=8, pair_g=9.8))
        c.save(f"perfdemo_chain_{n_pts}", run, spec, 40, None)
        OEng.Point.clear()


@scenario("g1_builders")
def sc_g1_builders(c):
    """M. G1 builders (gym/walker.py:138-353) run from the reference module itself (load_g1_walker), one of each in a
    ragged batch, observed with G1 getstat (midform 2: the position SUM), 2D, 40 steps."""
    c.fresh()
    G1 = load_g1_walker(c.args.ref, c.E)
    g1_names = ["leg2", "box", "box2", "balance", "balance2", "balance3", "intrian", "humanb", "insect", "box4",
                "leg", "hat"]
    crs = [getattr(G1, n)() for n in g1_names]
    for cr in crs:
        for e in list(cr.muscles) + list(cr.skeletons):
            e._string = 0
        for p in cr.phys:   # the batch stores masses as float32: balance2/3's 0.1 -> f32(0.1)
            p.m = float(np.float32(p.m))
    spec = spec_from_creatures(crs, None)
    acts = scenario_rng("g1_builders").uniform(-1, 1, (40, spec.N, int(spec.n_muscles.max()))).astype(f32)
    run = RefRun(c.E, c.OW, c.OE, crs, dict(in3d=0, midform=2, conmid=1), G1=G1)
    c.save("g1_builders", run, spec, 40, acts, extra={"g1_names": np.array(g1_names)})


class _Scene:
    def add_point(self, *a, **k):
        pass

    add_spring = add_point


def _env_recorder(g3env):
    class EnvRecorder:   # the state env.Environment.add_point / add_ding_point / add_spring write
        def __init__(self):
            self.points, self.ding_points, self.springs, self.scene = [], [], [], _Scene()

    for meth in ("add_point", "add_ding_point", "add_spring"):
        setattr(EnvRecorder, meth, getattr(g3env.Environment, meth))
    return EnvRecorder


G3_NAMES = [("leg2", {}), ("box", {}), ("balance1", {}), ("balance2", {}), ("balance3", {}), ("humanb", {}),
            ("insect", {}), ("insect8", {"legs": 8})]


@scenario("g3_builders")
def sc_g3_builders(c):
    """N. G3 builders (gym/optimized_walker/walker.py:377-639): their points and springs as the reference's own env
    methods record them (topology only).  tests/golden/topology/."""
    core, g3env, g3w = load_g3(c.args.ref)
    EnvRecorder = _env_recorder(g3env)
    topo = {}
    for n, kw in G3_NAMES:
        core.Point.points = []
        env = EnvRecorder()
        cr = getattr(g3w, n.rstrip("8") if n == "insect8" else n)(env, **kw)
        pts = cr.skeleton.points
        idx = {id(p): q for q, p in enumerate(pts)}
        topo[n + "_m"] = np.array([float(p.m) for p in pts])
        topo[n + "_pos"] = np.array([p.pos for p in pts], f32)
        topo[n + "_ding"] = np.array([isinstance(p, core.DingPoint) for p in pts], np.uint8)
        topo[n + "_springs"] = np.array([[idx[id(a)], idx[id(b)]] for a, b, x, k, st in env.springs], np.int32).reshape(-1, 2)
        topo[n + "_spring_x"] = np.array([x for a, b, x, k, st in env.springs], f32)
        topo[n + "_spring_k"] = np.array([k for a, b, x, k, st in env.springs], np.float64)
        topo[n + "_spring_string"] = np.array([st for a, b, x, k, st in env.springs], np.uint8)
        mus = cr.skeleton.muscles
        topo[n + "_muscles"] = np.array([[idx[id(mu.point1)], idx[id(mu.point2)]] for mu in mus], np.int32).reshape(-1, 2)
        topo[n + "_muscle_x"] = np.array([mu.x for mu in mus], f32)
        topo[n + "_muscle_power"] = np.array([mu.power for mu in mus], np.float64)
    c.write("g3_builders", topo, sub="topology")


@scenario("g3_physics")
def sc_g3_physics(c):
    """Q. G3 physics (gym/optimized_walker/env.py:135-184): the reference's own Environment.update_physics run on the
    G3 builders' own points and springs (one batch: every builder), with core.Point.run1 over the registry.  Gravity
    (1, -98, 0) and ground level -20 so the creatures land; every third spring a string and random initial
    velocities so the string and clamp paths both run.  150 steps.  tests/golden/g3/g3_physics.npz (state only: the
    G3 env has no observation or reward)."""
    core, g3env, g3w = load_g3(c.args.ref)
    EnvRecorder = _env_recorder(g3env)
    core.Point.points = []
    all_pts, all_springs, mass_off, edge_off = [], [], [0], [0]
    ei, ej, rest, kk, flags = [], [], [], [], []
    rng = scenario_rng("g3_physics")
    for n, kw in G3_NAMES:
        env = EnvRecorder()
        cr = getattr(g3w, n.rstrip("8") if n == "insect8" else n)(env, **kw)
        pts = cr.skeleton.points
        idx = {id(p): q for q, p in enumerate(pts)}
        for s_i, (a, b_, x, k, st) in enumerate(env.springs):
            st = bool(s_i % 3 == 2)
            all_springs.append((a, b_, x, k, st))
            ei.append(idx[id(a)]); ej.append(idx[id(b_)]); rest.append(np.float32(x)); kk.append(k)
            flags.append(1 if st else 0)
        for p in pts:
            if not isinstance(p, core.DingPoint):
                p.v[:] = rng.uniform(-5, 5, 3).astype(f32)
        all_pts.extend(pts)
        mass_off.append(len(all_pts)); edge_off.append(len(all_springs))
    ding = [p for p in all_pts if isinstance(p, core.DingPoint)]
    shim = types.SimpleNamespace(points=[p for p in all_pts if not isinstance(p, core.DingPoint)], ding_points=ding,
                                 springs=all_springs, gravity=np.array([1.0, -98.0, 0.0], f32), damping=0.99,
                                 air_resistance=0.01, ground=True, ground_level=-20.0, ground_restitution=0.8,
                                 friction=0.5, time_step=0.01, frame_count=0)
    core.Point.points = list(all_pts)
    g3in = dict(in_m=np.array([float(p.m) for p in all_pts], f32), in_pos=np.array([p.pos for p in all_pts], f32),
                in_vel=np.array([p.v for p in all_pts], f32), in_pinned=np.array([isinstance(p, core.DingPoint)
                                                                                  for p in all_pts], np.uint8),
                in_mass_off=np.array(mass_off, np.int32), in_edge_off=np.array(edge_off, np.int32),
                in_ei=np.array(ei, np.int32), in_ej=np.array(ej, np.int32), in_rest=np.array(rest, f32),
                in_k=np.array(kk, f32), in_c=np.zeros(len(rest), f32), in_flags=np.array(flags, np.uint8),
                in_n_muscles=np.zeros(len(G3_NAMES), np.int32), in_minl=np.zeros(0, f32),
                in_maxl=np.zeros(0, f32), in_stride=np.zeros(0, f32),
                param_g3_gravity=np.array([1.0, -98.0, 0.0]), param_g3_damping=np.array(0.99),
                param_g3_air=np.array(0.01), param_g3_ground=np.array(1), param_g3_ground_level=np.array(-20.0),
                param_g3_restitution=np.array(0.8), param_g3_friction=np.array(0.5), param_dt=np.array(0.01),
                param_spring_mode=np.array(2), param_in3d=np.array(1))
    outs = {"out_pos": [], "out_vel": [], "out_acc": []}
    for t in range(150):
        g3env.Environment.update_physics(shim)
        outs["out_pos"].append(np.array([p.pos for p in all_pts], f32))
        outs["out_vel"].append(np.array([p.v for p in all_pts], f32))
        outs["out_acc"].append(np.array([p.old_a for p in all_pts], f32))
    c.write("g3_physics", dict(**g3in, **{k: np.stack(v) for k, v in outs.items()},
                               g3_names=np.array([n for n, _ in G3_NAMES]), numpy_version=np.array(np.__version__)),
            sub="g3")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", nargs="*", default=None, help="run only the scenarios writing these fixtures")
    args = ap.parse_args(argv)
    E, OW, OE = load_reference(args.ref)
    c = Ctx(E, OW, OE, args)
    known = {n for names, _ in SCENARIOS for n in names}
    if args.only is not None and not set(args.only) <= known:
        raise SystemExit(f"unknown fixtures: {sorted(set(args.only) - known)}")
    for names, fn in SCENARIOS:
        if args.only is None or set(names) & set(args.only):
            fn(c)
    for name, size in c.written:
        print(f"{name:28s} {size:9d} B")


if __name__ == "__main__":
    main()
