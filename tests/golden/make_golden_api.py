#!/usr/bin/env python3
"""Golden vectors of the reference's drop-in API and done branches (this container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_api.py [--ref /root/reference]

Where make_golden.py drives the engine primitives directly, this script drives the reference's own env
objects, with SURVEY §8(c)'s mechanical fixes applied by overriding only the method that cannot run as written:

* ``gym/optimized_env.py`` ``PhysicsEnv``: its own ``__init__`` (which calls ``reset``), ``seed``, ``reset`` (global
  ``np.random.normal`` draws, :53-68), ``step`` (:70-92), ``_get_observation/_get_reward/_is_done/_get_info``
  (:184-248).  ``_run_physics`` (:140-178) raises TypeError as written (forces passed as lists,
  gym/engine.py:67); it is overridden by the same composition make_golden.RefRun.physics uses: engine.py springs
  (gym/engine.py:78-102) + the damping of gym/optimized_walker.py:92-106, then the env forces of :146-172 as
  float32 arrays, then the reference ``Point.run1``.  Creatures come from the reference's own
  ``create_balance_creature`` / ``create_box_creature`` (engine Points); ``make_env`` itself raises ImportError in
  the reference, so the env is constructed as make_env would construct it.
* ``gym/env.py`` ``Environment`` (G1): its own ``__init__`` (``random.gauss`` noise on every point, :21-26) and
  ``step(t)`` (:48-50: ``run()`` then ``Point.run1(t)``); ``run`` (:28-46) is overridden with the three fixes
  (forces as float32 arrays, ``.pos`` for ``.p``, the per-edge spring pass for the missing ``c.run1()``) and keeps
  the G1 friction force ``[v_x*deep*friction, 0, v_z*deep*friction]`` (:41).  Creatures: the G1 builders of
  gym/walker.py (make_golden.load_g1_walker).

Scenarios (tests/golden/api/*.npz):
  api_balance_2d       np.random.seed(123); PhysicsEnv(balance); seed(7); reset(); 60 steps of U(-1,1) actions
  api_box_3d_maxsteps  the same with Box-v0 in 3D, max_steps = 40, 45 steps: done from step 40 on
  api_settle           Balance-v0, dampk = 5, rand_sigma = 0, zero actions, 230 steps: every |v| < 0.1 after
                       step 100 -> done (gym/optimized_env.py:222-224)
  api_rollout_1000     Balance-v0 3D, zero actions, 1000 steps (SURVEY §7's 1,000-step zero-action rollout; done at
                       steps >= max_steps on the last step)
  g1_env               random.seed(5); G1 Environment([leg2, box, balance], in3d=True, randsigma=0.5, dampk=0.1);
                       50 step(t) calls with t cycling 0.01 / 0.005 / 0.02
Every output goes to --out (default tests/golden/api/); each scenario draws its actions from its own generator,
seeded by its name, so scenarios never shift one another.  (The performance_demo chain fixtures are engine-level:
make_golden.py.)
"""
from __future__ import annotations

import argparse
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402

f32 = np.float32


def env_forces(P, p, g1_friction=False):
    """gym/optimized_env.py:146-172 (gym/env.py:31-41) for one point, each force a float32 array."""
    p.forced(np.array([0, -P["g"], 0], dtype=f32))
    p.forced(np.asarray(-P["dampk"] * p.v, dtype=f32))
    if p.pos[1] - P["ground"] < 0:
        p.color = "red"; p.r = 3
        deep = p.pos[1] - P["ground"]
        p.forced(np.array([0, -P["groundk"] * deep, 0], dtype=f32))
        p.forced(np.array([0, -P["grounddamp"] * p.v[1], 0], dtype=f32))
        if g1_friction:   # gym/env.py:41
            p.forced(np.array([p.v[0] * deep * P["friction"], 0, p.v[2] * deep * P["friction"]], dtype=f32))
        else:             # gym/optimized_env.py:168-172
            ff = np.abs(deep) * P["friction"]
            p.forced(np.array([-p.v[0] * ff, 0, -p.v[2] * ff], dtype=f32))
    else:
        p.color = "black"; p.r = 1


def springs(OW, cr):
    """Creature.run's zero + spring pass with SURVEY §8(c) fix 3 (engine.py resilience + G2 damping)."""
    for p in cr.phys:
        p.zero()
    for e in list(cr.muscles) + list(cr.skeletons):
        e.p1.resilience(e.p2, e.x, e.k, False)
        OW.Skeleton(e.p1, e.p2, x=e.x, k=0, dampk=e.dampk).run()


def fixed_physics_env(E, OW, OE):
    class FixedPhysicsEnv(OE.PhysicsEnv):
        def _run_physics(self):   # gym/optimized_env.py:140-178 with the §8(c) fixes
            springs(OW, self.creature)
            P = dict(g=self.g, dampk=self.dampk, ground=self.ground, groundk=self.ground_k,
                     grounddamp=self.ground_damp, friction=self.friction)
            for p in self.creature.phys:
                env_forces(P, p)
            E.Point.run1(self.time_step)
    return FixedPhysicsEnv


def record_env(env, actions, T):
    """Drive reference env.step T times; record the API's return values and the point state."""
    pts = env.creature.phys
    out = {k: [] for k in ("obs", "reward", "done", "steps", "centroid", "energy", "pos", "vel", "acc")}
    for t in range(T):
        obs, reward, done, info = env.step(actions[t] if actions is not None else [])
        assert isinstance(obs, np.ndarray) and obs.dtype == np.float64
        assert isinstance(reward, np.float32), type(reward)
        assert isinstance(info["total_energy"], np.float32), type(info["total_energy"])
        out["obs"].append(obs); out["reward"].append(reward); out["done"].append(bool(done))
        out["steps"].append(info["steps"]); out["centroid"].append(info["centroid_position"])
        out["energy"].append(info["total_energy"])
        out["pos"].append([p.pos.copy() for p in pts]); out["vel"].append([p.v.copy() for p in pts])
        out["acc"].append([np.asarray(p.old_a).copy() for p in pts])
    return {"out_obs": np.array(out["obs"], np.float64), "out_reward": np.array(out["reward"], f32),
            "out_done": np.array(out["done"], np.uint8), "out_steps": np.array(out["steps"], np.int32),
            "out_centroid": np.array(out["centroid"], np.float64), "out_energy": np.array(out["energy"], f32),
            "out_pos": np.array(out["pos"], f32), "out_vel": np.array(out["vel"], f32),
            "out_acc": np.array(out["acc"], f32)}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "api"))
    ap.add_argument("--only", nargs="*", default=None, help="run only these scenarios")
    args = ap.parse_args(argv)
    want = (lambda name: args.only is None or name in args.only)
    E, OW, OE = MG.load_reference(args.ref)
    os.makedirs(args.out, exist_ok=True)
    FixedEnv = fixed_physics_env(E, OW, OE)
    written = []

    def fresh():
        E.Point.points = []
        E.Point.r_points = {}

    def save(name, blob):
        blob["numpy_version"] = np.array(np.__version__)
        path = os.path.join(args.out, name + ".npz")
        np.savez_compressed(path, **blob)
        written.append((name, os.path.getsize(path)))

    # ---- PhysicsEnv facade scenarios
    OW.Point = E.Point
    scen = [("api_balance_2d", "balance", dict(in3d=False), None, 60, "uniform"),
            ("api_box_3d_maxsteps", "box", dict(in3d=True), 40, 45, "uniform"),
            ("api_settle", "balance", dict(in3d=False, dampk=5, rand_sigma=0.0), None, 230, "zero"),
            ("api_rollout_1000", "balance", dict(in3d=True), None, 1000, "zero")]
    for name, creature, kw, max_steps, T, acts_kind in scen:
        if not want(name):
            continue
        fresh()
        cr = {"balance": OW.create_balance_creature, "box": OW.create_box_creature}[creature]()
        np.random.seed(123)
        env = FixedEnv(cr, **kw)                 # __init__ -> reset(): the first noise draw
        if max_steps is not None:
            env.max_steps = max_steps
        env.seed(7)
        obs0 = env.reset()                       # the second noise draw, after seed(7)
        A = len(cr.muscles)
        actions = (MG.scenario_rng(name).uniform(-1, 1, (T, A)).astype(f32) if acts_kind == "uniform"
                   else np.zeros((T, A), f32))
        rec = record_env(env, actions, T)
        blob = dict(env_id=np.array({"balance": "Balance-v0", "box": "Box-v0"}[creature]),
                    kwargs_in3d=np.array(int(kw.get("in3d", False))), kwargs_dampk=np.array(float(kw.get("dampk", 0))),
                    kwargs_rand_sigma=np.array(float(kw.get("rand_sigma", 0.1))),
                    max_steps=np.array(max_steps if max_steps is not None else 1000), np_seed_init=np.array(123),
                    env_seed=np.array(7), actions=actions, out_obs0=np.asarray(obs0, np.float64), **rec)
        if name == "api_rollout_1000":           # keep the fixture small: every 10th state, every step's scalars
            for k in ("out_obs", "out_pos", "out_vel", "out_acc", "out_centroid"):
                blob[k] = blob[k][9::10]
        save(name, blob)
        print(name, "done steps:", np.nonzero(rec["out_done"])[0][:3] + 1)

    # ---- G1 Environment (gym/env.py) with G1 creatures
    if want("g1_env"):
        g1_env(args, E, OW, fresh, save)
    for name, size in written:
        print(f"{name:22s} {size:9d} B")


def g1_env(args, E, OW, fresh, save):
    fresh()
    import gym.env as GE
    G1 = MG.load_g1_walker(args.ref, E)

    class FixedG1Env(GE.Environment):
        def run(self):                           # gym/env.py:28-46 with the §8(c) fixes
            P = dict(g=self.g, dampk=self.dampk, ground=self.ground, groundk=self.groundk,
                     grounddamp=self.grounddamp, friction=self.friction)
            for c in self.creatures:
                springs(OW, c)
                for p in c.phys:
                    env_forces(P, p, g1_friction=True)

    names = ["leg2", "box", "balance"]
    crs = [getattr(G1, n)() for n in names]
    random.seed(5)
    env = FixedG1Env(crs, in3d=True, dampk=0.1, randsigma=0.5)
    pts = [p for c in crs for p in c.phys]
    vel0 = np.array([p.v.copy() for p in pts], f32)
    ts = [0.01, 0.005, 0.02] * 17
    ts = ts[:50]
    pos, vel, acc = [], [], []
    for t in ts:
        env.step(t)
        pos.append([p.pos.copy() for p in pts]); vel.append([p.v.copy() for p in pts])
        acc.append([np.asarray(p.old_a).copy() for p in pts])
    save("g1_env", dict(g1_names=np.array(names), random_seed=np.array(5), in3d=np.array(1), dampk=np.array(0.1),
                        randsigma=np.array(0.5), ts=np.array(ts), out_vel0=vel0, out_pos=np.array(pos, f32),
                        out_vel=np.array(vel, f32), out_acc=np.array(acc, f32)))


if __name__ == "__main__":
    main()
