"""G1 ``Environment`` (gym/env.py:9-50) on the HIP stepper.

``Environment(creaturelist, in3d, g, dampk, groundhigh, groundk, grounddamp, friction, randsigma)``
adds ``random.gauss(0, randsigma)`` to v_x, v_y (and v_z in 3D) of every point at construction
(gym/env.py:21-26 — Python's ``random`` module, drawn in the same order here), and ``step(t)``
applies the env forces and integrates with dt = t (gym/env.py:48-50).  The reference's broken
``c.run1()`` call (gym/env.py:30) is the spring pass of SURVEY §0.1 step 3; the ground friction is the G1
form ``[v_x*deep*friction, 0, v_z*deep*friction]`` (gym/env.py:41, friction_mode 1), which rounds differently
from the G2 env's.  Pinned by tests/golden/api/g1_env.npz (the reference's own Environment).
"""
from __future__ import annotations

import random

import numpy as np

from .optimized_env import Environment as _CompatEnvironment


class Environment(_CompatEnvironment):
    _friction_mode = 1   # gym/env.py:41: [v_x*deep*friction, 0, v_z*deep*friction]

    def reset(self) -> np.ndarray:
        self._sync_params()
        P = self._env.batch.P
        noise = np.zeros((P, 3), np.float32)
        for q in range(P):
            noise[q, 0] = random.gauss(0, self.sigma)
            noise[q, 1] = random.gauss(0, self.sigma)
            if self.in3d:
                noise[q, 2] = random.gauss(0, self.sigma)
        obs = self._env.reset(noise=noise)
        self._cache = None
        return self._obs_np(obs, int(self._env.obs_len[0]))


__all__ = ["Environment"]
