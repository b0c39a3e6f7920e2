"""walker_gym_amd — MI355X-native batched walker physics stepper (the hot path of bluemoon-o2/walker-gym).

Product path: BatchedPhysicsEnv (walker_gym_amd.batched_env) over libwalker_hip.so (C ABI in
include/walker_hip.h, HIP kernels for gfx950).  Drop-in facades of the reference API:
  walker_gym_amd.engine        Point, Config, to_data, DingPoint            (gym/engine.py)
  walker_gym_amd.walker        Muscle, Skeleton, Creature, create_*_creature (gym/optimized_walker.py)
  walker_gym_amd.optimized_env PhysicsEnv, make_env, Environment            (gym/optimized_env.py)
  walker_gym_amd.env           Environment (G1 step(t) API)                  (gym/env.py)
  walker_gym_amd.snapshot      state.pkl read/write without unpickling       (gym/engine.py:199-212)
Importing the package needs no GPU; stepping does (no CPU fallback).
"""
from .engine import Config, DingPoint, Point, to_data  # noqa: F401
from .walker import (Creature, Muscle, Skeleton, balance_spec, box_spec, create_balance_creature,  # noqa: F401
                     create_box_creature, creatures_to_spec)

__version__ = "0.1.0"


def __getattr__(name):
    # torch-dependent modules load lazily so `import walker_gym_amd` stays light
    if name in ("BatchedPhysicsEnv", "EnvParams"):
        from . import batched_env
        return getattr(batched_env, name)
    if name in ("PhysicsEnv", "make_env"):
        from . import optimized_env
        return getattr(optimized_env, name)
    raise AttributeError(name)
