"""Shared replay of tests/golden/api fixtures (not a test module): the reset-noise sequences the reference's
PhysicsEnv.reset / G1 Environment.__init__ draw, and the creatures of each fixture in this repo's API."""
import random

import numpy as np


def physicsenv_noise(P: int, sigma: float, in3d: bool, np_seed: int, env_seed: int):
    """gym/optimized_env.py:53-68: per point np.random.normal(0, sigma) for v_x, v_y (and v_z in 3D), in point
    order; PhysicsEnv.__init__ draws once after np.random.seed(np_seed), reset() after env.seed(env_seed) again.
    The Python float is weakly cast to float32 by `p.v[0] += ...` (NEP 50), so float32 noise is exact."""
    out = []
    for seed in (np_seed, env_seed):
        np.random.seed(seed)
        n = np.zeros((P, 3), np.float32)
        for q in range(P):
            n[q, 0] = np.random.normal(0, sigma)
            n[q, 1] = np.random.normal(0, sigma)
            if in3d:
                n[q, 2] = np.random.normal(0, sigma)
        out.append(n)
    return out


def g1_noise(P: int, sigma: float, in3d: bool, seed: int):
    """gym/env.py:21-26: random.gauss(0, sigma) for v_x, v_y (v_z in 3D) of every point, after random.seed(seed)."""
    random.seed(seed)
    n = np.zeros((P, 3), np.float32)
    for q in range(P):
        n[q, 0] = random.gauss(0, sigma)
        n[q, 1] = random.gauss(0, sigma)
        if in3d:
            n[q, 2] = random.gauss(0, sigma)
    return n


def api_creature(env_id: str):
    from walker_gym_amd.walker import create_balance_creature, create_box_creature
    return {"Balance-v0": create_balance_creature, "Box-v0": create_box_creature}[env_id]()


def g1_creatures(names):
    from walker_gym_amd.topologies import build_creature
    return [build_creature(str(n), generation=1) for n in names]
