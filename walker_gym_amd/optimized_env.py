"""PhysicsEnv / make_env / Environment — the reference's gym-style API on the HIP stepper.

Drop-in for gym/optimized_env.py:8-334: same constructor arguments and defaults, same return types:
  reset() -> np.ndarray[D] (float64, like ``np.array(getstat_list)``)
  step(action) -> (obs np.ndarray[D], reward np.float32, done bool, info dict)
  info = {'steps': int, 'centroid_position': [x, y, z], 'total_energy': np.float32}
The creature is packed into a one-walker BatchedPhysicsEnv; each step is one kernel launch.  For
throughput, batch many walkers with walker_gym_amd.batched_env.BatchedPhysicsEnv instead.

Reset noise: the reference draws ``np.random.normal(0, sigma)`` per mass for v_x, v_y (and v_z in 3D),
in mass order (gym/optimized_env.py:56-62); this facade draws the SAME sequence from numpy's global
RNG and injects it, so ``np.random.seed(s)`` / ``env.seed(s)`` reproduces the reference bit for bit.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from .batched_env import BatchedPhysicsEnv
from .walker import Creature, create_balance_creature, create_box_creature, creatures_to_spec


class PhysicsEnv:
    metadata = {"render.modes": [], "video.frames_per_second": 60}

    def __init__(self, creature: Creature, in3d: bool = False, g: float = 100, dampk: float = 0,
                 ground_high: float = 0, ground_k: float = 1000, ground_damp: float = 100,
                 friction: float = 100, rand_sigma: float = 0.1, device=None):
        self.creature = creature
        self.in3d = in3d
        self.g, self.dampk, self.ground = g, dampk, ground_high
        self.ground_k, self.ground_damp, self.friction = ground_k, ground_damp, friction
        self.sigma = rand_sigma
        self.time_step = 0.01            # gym/optimized_env.py:42
        self.max_steps = 1000            # :44
        self._creatures = [creature] if creature is not None else []
        self._env = self._make_env(device)
        self._bind_points()
        self.reset()

    # ---------------------------------------------------------------- plumbing
    def _make_env(self, device):
        spec = creatures_to_spec(self._creatures)
        return BatchedPhysicsEnv(spec, device=device, g=self.g, dampk=self.dampk, ground=self.ground,
                                 groundk=self.ground_k, grounddamp=self.ground_damp, friction=self.friction,
                                 dt=self.time_step, in3d=self.in3d, max_steps=self.max_steps)

    def _bind_points(self):
        q = 0
        for cr in self._creatures:
            for p in cr.phys:
                p._env, p._index = self, q
                q += 1
        self._cache = None

    def _host_state(self):
        if self._cache is None:
            b = self._env.batch
            self._cache = {"pos": b.caller("pos").cpu().numpy(), "v": b.caller("vel").cpu().numpy(),
                           "old_a": b.caller("acc").cpu().numpy()}
        return self._cache

    def _point_state(self, index: int, name: str) -> np.ndarray:
        return self._host_state()[name][index].copy()

    def _set_point_state(self, index: int, name: str, value) -> None:
        b = self._env.batch
        t = {"pos": b.pos, "v": b.vel}[name]
        t[b.stored_mass(index)] = torch.as_tensor(np.asarray(value, np.float32), device=t.device)
        self._cache = None

    _friction_mode = 0   # gym/optimized_env.py:168-172; the G1 Environment (walker_gym_amd.env) uses gym/env.py:41

    def _param_values(self):
        return dict(g=self.g, dampk=self.dampk, ground=self.ground, groundk=self.ground_k,
                    grounddamp=self.ground_damp, friction=self.friction, dt=self.time_step, in3d=bool(self.in3d),
                    max_steps=self.max_steps, friction_mode=self._friction_mode)

    def _sync_params(self, force: bool = True):
        """Push the env's attributes (the reference keeps them as plain attributes a caller may change between
        steps, e.g. ``env.max_steps``) to the batched env; without ``force`` only when one of them changed."""
        vals = self._param_values()
        if force or vals != getattr(self, "_synced", None):
            self._env.set_params(**vals)
            self._synced = vals

    @staticmethod
    def _obs_np(obs: torch.Tensor, n: int) -> np.ndarray:
        return obs[0, :n].cpu().numpy().astype(np.float64)

    # ---------------------------------------------------------------- gym API
    def reset(self) -> np.ndarray:
        """gym/optimized_env.py:53-68 (a = 0, v += N(0, sigma), steps = 0)."""
        self._sync_params()
        P = self._env.batch.P
        noise = np.zeros((P, 3), np.float32)
        for q in range(P):
            noise[q, 0] = np.random.normal(0, self.sigma)
            noise[q, 1] = np.random.normal(0, self.sigma)
            if self.in3d:
                noise[q, 2] = np.random.normal(0, self.sigma)
        obs = self._env.reset(noise=noise)
        self._cache = None
        return self._obs_np(obs, int(self._env.obs_len[0]))

    @property
    def steps(self) -> int:
        return int(self._env.steps[0].item())

    def step(self, action: Union[List[float], np.ndarray]) -> Tuple[np.ndarray, np.float32, bool, Dict[str, Any]]:
        """gym/optimized_env.py:70-92: act -> physics -> steps += 1 -> obs, reward, done, info."""
        a = np.asarray(action if action is not None else [], dtype=np.float32).reshape(1, -1)
        self._sync_params(force=False)
        obs, rew, done, info = self._env.step(a if a.shape[1] else None)
        self._cache = None
        c = info["centroid_position"][0].cpu().numpy()
        return (self._obs_np(obs, int(self._env.obs_len[0])), np.float32(rew[0].item()), bool(done[0].item()),
                {"steps": int(info["steps"][0].item()), "centroid_position": [float(v) for v in c],
                 "total_energy": np.float32(info["total_energy"][0].item())})

    def render(self, mode: str = "human"):
        raise NotImplementedError("rendering is out of scope for the MI355X stepper (SURVEY §2 row 8)")

    def close(self) -> None:
        pass

    def seed(self, seed: Optional[int] = None) -> List[int]:
        """gym/optimized_env.py:130-138: seeds numpy's global RNG (the reset noise source)."""
        np.random.seed(seed)
        return [seed] if seed is not None else []

    def get_action_space(self) -> Dict[str, Any]:
        return {"shape": (len(self.creature.muscles),), "type": "continuous", "low": -1.0, "high": 1.0}

    def get_observation_space(self) -> Dict[str, Any]:
        return {"shape": (int(self._env.obs_len[0]),), "type": "continuous", "low": -np.inf, "high": np.inf}


def make_env(env_id: str, **kwargs) -> PhysicsEnv:
    """gym/optimized_env.py:273-294."""
    env_id = env_id.lower()
    if env_id == "balance-v0":
        return PhysicsEnv(create_balance_creature(), **kwargs)
    if env_id == "box-v0":
        return PhysicsEnv(create_box_creature(), **kwargs)
    raise ValueError(f"Unknown environment ID: {env_id}")


class Environment(PhysicsEnv):
    """Legacy multi-creature API (gym/env.py:9-50, compat class gym/optimized_env.py:298-334):
    every creature in ``creaturelist`` is stepped (batched, one launch) by ``step(t)`` with dt = t."""

    def __init__(self, creaturelist, in3d=False, g=100, dampk=0, groundhigh=0, groundk=1000, grounddamp=100,
                 friction=100, randsigma=0.1, device=None):
        self.creatures = list(creaturelist)
        self.creature = self.creatures[0] if self.creatures else None
        self.in3d, self.g, self.dampk, self.ground = in3d, g, dampk, groundhigh
        self.ground_k, self.ground_damp, self.friction, self.sigma = groundk, grounddamp, friction, randsigma
        self.time_step = 0.01
        self.max_steps = 1000
        self._creatures = self.creatures
        self._env = self._make_env(device)
        self._bind_points()
        self.reset()

    def run(self) -> None:
        """One force pass + integration with the current time step (gym/env.py:28-46 + run1)."""
        self.step(self.time_step)

    def step(self, t):  # type: ignore[override]
        """gym/env.py:48-50: forces, then Point.run1(t)."""
        self.time_step = float(t)
        self._sync_params(force=False)
        self._env.step(None)
        self._cache = None
