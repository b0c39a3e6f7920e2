#!/usr/bin/env python3
"""BASELINE.json config 0: one walker stepped through the reference's gym-style API
(gym/optimized_env.py:53-92: reset -> step(action) -> (obs, reward, done, info)), here on the MI355X
stepper (one launch per step; the reference's own demo.py is empty).

    python demo.py [--env Balance-v0|Box-v0] [--steps 200] [--seed 0] [--g1 leg2]

``--g1 NAME`` runs one of the G1 builders (gym/walker.py:138-353, walker_gym_amd.topologies) through the
legacy ``Environment(...).step(t)`` API (gym/env.py:48-50) instead.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="Balance-v0")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--g1", default=None, help="a gym/walker.py topology run through gym/env.py Environment")
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    if a.g1:
        from walker_gym_amd.env import Environment
        from walker_gym_amd.topologies import build_creature
        cr = build_creature(a.g1, generation=1)
        env = Environment([cr], in3d=False)
        for t in range(a.steps):
            env.step(0.01)                              # gym/env.py:48-50 (no actions in the G1 loop)
        print(f"{a.g1}: {a.steps} steps, centroid {np.mean([p.pos for p in cr.phys], axis=0)}")
        return
    from walker_gym_amd.optimized_env import make_env
    env = make_env(a.env, in3d=False)
    env.seed(a.seed)
    obs = env.reset()
    total = 0.0
    for t in range(a.steps):
        obs, reward, done, info = env.step(rng.uniform(-1, 1, env.get_action_space()["shape"][0]))
        total += float(reward)
        if done:
            break
    print(f"{a.env}: {info['steps']} steps, return {total:.3f}, centroid {info['centroid_position']}, "
          f"energy {info['total_energy']:.3f}, obs dim {obs.shape[0]}")


if __name__ == "__main__":
    main()
