"""BatchedPhysicsEnv — N independent walkers stepped by one HIP launch per env step.

The batched form of the reference's gym-style API (gym/optimized_env.py:8-269):
  reset(noise=None, mask=None)        -> obs [N, D]                     (PhysicsEnv.reset :53-68)
  step(action [N, A])                 -> obs, reward [N], done [N], info (PhysicsEnv.step :70-92)
  rollout(actions [T, N, A])          -> obs [T, N, D], reward [T, N], done [T, N]   (one C call)
  observe()                           -> obs, reward, done, info for the current state
Environment parameters keep the reference's names and defaults (PhysicsEnv.__init__ :15-17).
obs rows are Creature.getstat (gym/optimized_walker.py:129-162), zero-padded to D = max row length
for ragged batches (``obs_len`` gives each walker's length).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, asdict
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from .device import DeviceBatch
from .layout import HostLayout, pack


@dataclass
class EnvParams:
    """PhysicsEnv / Environment constructor parameters + getstat options (reference defaults)."""
    g: float = 100.0
    dampk: float = 0.0
    ground: float = 0.0           # ground_high / groundhigh
    groundk: float = 1000.0       # ground_k
    grounddamp: float = 100.0     # ground_damp
    friction: float = 100.0
    dt: float = 0.01              # PhysicsEnv.time_step (optimized_env.py:42)
    in3d: bool = False
    max_steps: int = 1000         # optimized_env.py:44
    pk: float = 1.0
    vk: float = 1.0
    ak: float = 1.0
    mk: float = 1.0
    midform: int = 1              # 1: minus the mean (G2 getstat); 2: minus the SUM (G1 getstat); 0: raw
    conmid: bool = False
    spring_mode: int = 0          # 0: engine.py resilience + damping; 1: G2 optimized_walker as written
    action_mode: int = 0          # 0: Muscle.act; 1: Muscle.actdisp
    integrator: int = 1           # 1: Point.run1 (what the envs call); 2: Point.run2 (gym/engine.py:180-190)
    pair_mode: int = 0            # bitmask, per walker after the springs: 1 Point.gravity (gym/engine.py:128-137),
                                  # 2 Point.coulomb (:139-147), 4 Point.bounce (:114-125), in that order
    pair_g: float = 9.8           # Config.g of the gravity pass (gym/engine.py:12)
    pair_k: float = 8.99e9        # Config.k of the coulomb pass (gym/engine.py:11)
    pair_e: float = 16e-20        # Point.e of every point without a spec charge (Config.e, gym/engine.py:10)
    bounce_k: float = 100.0       # Point.bounce(k) (gym/engine.py:114)
    # spring_mode 2: the G3 engine (gym/optimized_walker/env.py:10-14 defaults, update_physics :135-184)
    g3_gravity: tuple = (0.0, -9.8, 0.0)
    g3_damping: float = 0.99
    g3_air: float = 0.01
    g3_ground_level: float = -50.0
    g3_restitution: float = 0.8
    g3_friction: float = 0.5
    g3_ground: int = 1
    friction_mode: int = 0        # 0: gym/optimized_env.py:168-172 friction; 1: the G1 env's (gym/env.py:41)

    def to_struct(self) -> _lib.WgParams:
        d = asdict(self)
        if d["integrator"] in ("run1", "run2"):
            d["integrator"] = int(d["integrator"][-1])
        if int(d["integrator"]) not in (0, 1, 2):
            raise ValueError("integrator must be 1 ('run1') or 2 ('run2')")
        gv = tuple(float(x) for x in d.pop("g3_gravity"))
        if len(gv) != 3:
            raise ValueError("g3_gravity must have 3 components")
        return _lib.WgParams(g3_gravity=(C.c_double * 3)(*gv),
                             **{k: (int(v) if k in ("in3d", "max_steps", "midform", "conmid", "spring_mode",
                                                    "action_mode", "integrator", "pair_mode", "g3_ground",
                                                    "friction_mode")
                                    else float(v)) for k, v in d.items()})


def require_tensor(t, name: str, device, dtype, shape=None) -> None:
    """Refuse a tensor whose raw pointer the kernel cannot use as given: another device (host memory or another
    GPU), another dtype, a non-contiguous layout or a wrong shape.  Raises ValueError before any launch."""
    if not isinstance(t, torch.Tensor):
        raise ValueError(f"{name} must be a torch tensor on {device}")
    # (on the per-call path of run(): `torch.device.__ne__` and tuple(t.shape) cost microseconds each, == does not)
    if not (t.device == (device if isinstance(device, torch.device) else torch.device(device))):
        raise ValueError(f"{name} is on {t.device}, the batch is on {device}")
    if t.dtype != dtype:
        raise ValueError(f"{name} has dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and not (t.shape == (shape if isinstance(shape, tuple) else tuple(shape))):
        raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")


class WalkerGraph:
    """A captured run() (BatchedPhysicsEnv.graph).  The graph holds raw pointers to the env's state and output
    tensors and the parameters as they were at capture: set_params / a reallocation of the outputs / enabling
    radii bump the env's generation, and replay() of a graph captured before that raises instead of writing
    into freed memory or silently stepping with stale parameters."""

    def __init__(self, env: "BatchedPhysicsEnv", graph, actions, info: bool = True):
        self._env, self._graph, self._gen = env, graph, env._generation
        self.actions = actions            # kept alive: the graph reads it on every replay
        # the replayed steps write info['steps'] in caller order (env.steps_out) only when captured with info
        self._writes_steps = bool(info) and env.steps_out is not None
        self._stale = frozenset() if info else frozenset({"centroid_position", "total_energy", "momentum", "nonfinite"})

    def replay(self) -> None:
        env = self._env
        if env._generation != self._gen:
            raise RuntimeError("stale WalkerGraph: the env's parameters or buffers changed after capture; "
                               "capture a new graph")
        self._graph.replay()
        # the batch's step counters moved: steps_out is current only if the graph wrote it (a graph
        # captured with info=False left a step()'s steps_out looking valid)
        env._steps_at = env.batch.version if self._writes_steps else -1
        env._stale = self._stale


class _RangeGraphs:
    """One captured graph per walker range and the stream it replays on (graph(), policy_loop(graph=True)): replay()
    forks the ranges from the calling stream, replays each on its own stream and joins them back.  (One graph holding
    the ranges as parallel branches replayed them serially on ROCm: 36.4 against 33.5 us per canonical step direct,
    profiles/r05y_bench_graph.json.)"""

    def __init__(self, parts, cur):
        self.parts, self._cur = parts, cur

    def replay(self) -> None:
        # range 0 replays on the calling stream itself (a single range needs no fork), the others on their own streams
        cur = torch.cuda.current_stream(self._cur.device)
        for g, st in self.parts[1:]:
            st.wait_stream(cur)
        for g, st in self.parts[1:]:
            with torch.cuda.stream(st):
                g.replay()
        self.parts[0][0].replay()
        for g, st in self.parts[1:]:
            cur.wait_stream(st)


class PreparedRun:
    """run()'s C call with its arguments already built (BatchedPhysicsEnv.prepare_run): calling it issues the prepared
    steps again.  Like a WalkerGraph it refuses to run once the env's parameters or buffers have changed."""

    def __init__(self, env: "BatchedPhysicsEnv", entry: str, fn, args, keep, steps_valid: bool, stale: set,
                 thunk=None):
        self._env, self._gen, self._struct = env, env._generation, env.batch.struct
        self._entry, self._fn, self._args, self._keep, self._thunk = entry, fn, args, keep, thunk
        self._steps_valid, self._stale = steps_valid, frozenset(stale)

    def __call__(self) -> None:
        env = self._env
        if env._generation != self._gen or env.batch.struct is not self._struct:
            raise RuntimeError("stale PreparedRun: the env's parameters or buffers changed after prepare_run")
        if self._thunk is not None:
            self._thunk(*self._args)
        else:
            rc = self._fn(*self._args)
            if rc:
                _lib.check(rc, self._entry)
        env._steps_at = env.batch.version if self._steps_valid else -1
        env._stale = self._stale


class BatchedPhysicsEnv:
    def __init__(self, spec_or_layout, device=None, rand_sigma: float = 0.0, seed: Optional[int] = None,
                 contact: bool = True, info_extras: bool = False, **params):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
        if device is None:
            raise RuntimeError("BatchedPhysicsEnv needs a ROCm GPU (libwalker_hip.so); there is no CPU path")
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        _lib.load()   # fail loudly before allocating anything
        self.params = EnvParams(**params)
        self.sigma = float(rand_sigma)
        host = spec_or_layout if isinstance(spec_or_layout, HostLayout) else pack(spec_or_layout)
        self.batch = DeviceBatch(host, device, contact=contact, wave_ok=self._wave_ok())
        if int(self.params.pair_mode) & 4:
            self.batch.enable_radius()
        self.device = device
        self.N = host.N
        self.obs_len = host.obs_len(self.params.in3d, self.params.conmid)
        self.obs_dim = int(self.obs_len.max())
        self._pstruct = self.params.to_struct()
        self._gen = torch.Generator(device=device)
        if seed is not None:
            self._gen.manual_seed(int(seed))
        self._generation = 0
        self._stale = frozenset()   # info() keys the last run() did not write (record buffers / info=False)
        # opt-in info (ABI 10): info['momentum'] (Point.momentum per walker, gym/engine.py:160-166) and
        # info['nonfinite'] (a walker whose state holds an inf / NaN; done is left as the reference computes it)
        self._extras = bool(info_extras)
        self._alloc_outputs()
        # the side streams of the default walker ranges, created now: a stream's hardware queue is bound when it is
        # created, and a process has few of them (GPU_MAX_HW_QUEUES = 4).  Created after an RCCL communicator
        # (whose streams take queues of their own) a side stream can share the calling stream's queue, which
        # serialises the ranges: 52.8 against 37.5 us per canonical step (profiles/r03a_bench_nccl1.json).
        self._side = []
        self.reserve_streams(self._lanes(None))

    @classmethod
    def from_topologies(cls, topologies, n_envs: int, device=None, **params) -> "BatchedPhysicsEnv":
        """SURVEY §8(b)'s BatchedPhysicsEnv(topologies, n_envs, device, **EnvParams): n_envs walkers split into
        contiguous, near-equal blocks, one per topology in order (uniform when there is one).  A topology is
        a Creature (walker_gym_amd.walker / .topologies builders) or an env id of make_env ('Balance-v0',
        'Box-v0', gym/optimized_env.py:273-294; unknown ids raise ValueError as there)."""
        from .walker import (Creature, concat_specs, create_balance_creature, create_box_creature,
                             creatures_to_spec, replicate_spec)
        if isinstance(topologies, (str, Creature)):
            topologies = [topologies]
        topologies = list(topologies)
        if not topologies or n_envs < len(topologies):
            raise ValueError("need at least one topology and one env per topology")
        specs = []
        for t, topo in enumerate(topologies):
            if isinstance(topo, str):
                tid = topo.lower()
                if tid == "balance-v0":
                    topo = create_balance_creature()
                elif tid == "box-v0":
                    topo = create_box_creature()
                else:
                    raise ValueError(f"Unknown environment ID: {topo}")
            count = n_envs // len(topologies) + (1 if t < n_envs % len(topologies) else 0)
            specs.append(replicate_spec(creatures_to_spec([topo]), count))
        return cls(specs[0] if len(specs) == 1 else concat_specs(specs), device=device, **params)

    # ------------------------------------------------------------------ plumbing
    def _alloc_outputs(self):
        self._generation += 1
        N, D, dv = self.N, self.obs_dim, self.device
        self.obs = torch.zeros((N, D), dtype=torch.float32, device=dv)
        self.reward = torch.zeros(N, dtype=torch.float32, device=dv)
        # bool storage: the kernel writes 0 / 1 bytes, so step() returns it as is (no conversion launch per step)
        self.done = torch.zeros(N, dtype=torch.bool, device=dv)
        self.centroid = torch.zeros((N, 3), dtype=torch.float32, device=dv)
        self.energy = torch.zeros(N, dtype=torch.float32, device=dv)
        # info['steps'] of a permuted (ragged) batch in the caller's order, written by the step kernels themselves
        # (wg_outputs.steps) so that step() needs no gather; valid while _steps_at == the batch's state version
        self.steps_out = torch.zeros(N, dtype=torch.int32, device=dv) if self.batch._perm else None
        self._steps_at = -1
        self.momentum = torch.zeros((N, 3), dtype=torch.float32, device=dv) if self._extras else None
        self.nonfinite = torch.zeros(N, dtype=torch.bool, device=dv) if self._extras else None

    def enable_info_extras(self) -> None:
        """Start producing info['momentum'] and info['nonfinite'] every step (one small per-walker pass after the
        step kernel).  The other output tensors stay the same objects; graphs captured before this raise on replay."""
        if not self._extras:
            # only the two new buffers (reallocating every output silently detached the tensors a caller
            # still held from step()); the generation bump makes cached plans and graphs rebuild / refuse
            self._extras = True
            self.momentum = torch.zeros((self.N, 3), dtype=torch.float32, device=self.device)
            self.nonfinite = torch.zeros(self.N, dtype=torch.bool, device=self.device)
            self._generation += 1

    def _outputs(self, obs=None, reward=None, done=None, centroid=None, energy=None, obs_step=0, out_step=0,
                 pad_clean=False, steps=None, nonfinite=None, momentum=None):
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        return _lib.WgOutputs(obs=p(obs), obs_stride=self.obs_dim, reward=p(reward), done=p(done),
                              centroid=p(centroid), energy=p(energy), obs_step=obs_step, out_step=out_step,
                              obs_pad_clean=int(pad_clean), steps=p(steps), nonfinite=p(nonfinite),
                              momentum=p(momentum))

    @staticmethod
    def _range_outputs(o, w0: int):
        """The WgOutputs of a uniform walker range starting at walker w0: o's pointers advanced by w0 rows (every output
        is walker-major: obs rows of obs_stride floats, f32 reward / energy, 1-byte done / nonfinite, int32 steps,
        3 x f32 centroid / momentum).  Pointer arithmetic instead of tensor slices: no per-call tensor views."""
        def adv(ptr, nbytes):
            return None if not ptr else C.c_void_p(ptr + nbytes)
        return _lib.WgOutputs(obs=adv(o.obs, 4 * w0 * o.obs_stride), obs_stride=o.obs_stride,
                              reward=adv(o.reward, 4 * w0), done=adv(o.done, w0), centroid=adv(o.centroid, 12 * w0),
                              energy=adv(o.energy, 4 * w0), obs_step=o.obs_step, out_step=o.out_step,
                              obs_pad_clean=o.obs_pad_clean, steps=adv(o.steps, 4 * w0),
                              nonfinite=adv(o.nonfinite, w0), momentum=adv(o.momentum, 12 * w0))

    def _extra_out(self, w0: int = 0, w1: Optional[int] = None) -> dict:
        """The opt-in info outputs of walkers [w0, w1) (or none)."""
        if not self._extras:
            return {}
        w1 = self.N if w1 is None else w1
        return {"nonfinite": self.nonfinite[w0:w1], "momentum": self.momentum[w0:w1]}

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def set_params(self, **kw):
        for k, v in kw.items():
            if not hasattr(self.params, k):
                raise AttributeError(k)
            setattr(self.params, k, v)
        obs_len = self.batch.host.obs_len(self.params.in3d, self.params.conmid)
        if not np.array_equal(obs_len, self.obs_len):   # new row lengths: fresh zero-padded outputs
            self.obs_len = obs_len
            self.obs_dim = int(obs_len.max())
            self._alloc_outputs()
        if int(self.params.pair_mode) & 4:
            self.batch.enable_radius()
        if self._needs_plan() and self.batch.wave_ok != self._wave_ok():
            self.batch.replan(self._wave_ok())   # the plan kind follows the parameters (DeviceBatch.replan)
        self._pstruct = self.params.to_struct()
        self._generation += 1   # graphs captured before this replay stale parameters: WalkerGraph refuses them

    def _wave_ok(self) -> bool:
        """The parameters can run on the barrier-free wave kernels (engine.py springs, no pair forces)."""
        return int(self.params.spring_mode) == 0 and int(self.params.pair_mode) == 0

    def _needs_plan(self) -> bool:
        """Batches whose launch plan depends on the parameters: ragged, or uniform with M not dividing 64."""
        M = self.batch.M
        return bool(self.batch.host.ragged) or not (4 <= M <= 64 and 64 % M == 0)

    def resident_ok(self) -> bool:
        """wg_rollout keeps the walkers in registers across steps (one launch for every step) for this batch and
        these parameters: uniform, M | 64, engine.py springs, no pair forces (otherwise it steps like wg_step)."""
        M = self.batch.M
        return (not self.batch.ragged and 4 <= M <= 64 and 64 % M == 0 and self._wave_ok()
                and os.environ.get("WG_LEAN", "1") != "0")

    def _check_action(self, action):
        if action is None:
            return None, 0
        if (isinstance(action, torch.Tensor) and action.dim() == 2 and action.dtype == torch.float32
                and action.device == self.device and action.shape[0] == self.N and action.is_contiguous()):
            return action, action.shape[1]                      # the closed-loop fast path: used as given
        if not isinstance(action, torch.Tensor):
            action = torch.as_tensor(np.asarray(action, dtype=np.float32))
        action = action.to(self.device, torch.float32)
        if action.dim() == 1 and self.N == 1:
            action = action[None]
        if action.dim() != 2 or action.shape[0] != self.N:
            raise ValueError(f"action must be [N={self.N}, A], got {tuple(action.shape)}")
        return action.contiguous(), action.shape[1]

    # ------------------------------------------------------------------ API
    def step(self, action=None):
        """One env step for all walkers: act -> physics -> run1 -> obs/reward/done/info: one launch per walker range
        (the default ranges, forked from and joined back to the calling stream inside one wg_step_ranges call).  The
        C arguments of every range are built once and cached (_step_plan): a closed-loop caller pays one ctypes
        call per step."""
        act, cols = self._check_action(action)
        plan = self._step_plan(cols if act is not None else -1)
        cur = torch.cuda.current_stream(self.device)
        rng = plan["ranges"]
        rng[0].stream = cur.cuda_stream
        rc = plan["fn"](rng, plan["n"], self._pref, act.data_ptr() if act is not None else None, cols, cols,
                        plan["events"])
        if rc:
            _lib.check(rc, "wg_step_ranges")
        self._steps_at = self.batch.version
        self._stale = frozenset()
        if act is not None and plan["n"] > 1 and not torch.cuda.is_current_stream_capturing():
            for st in plan["side"]:
                act.record_stream(st)   # the allocator must not recycle the actions before the side streams read them
        return self.obs, self.reward, self.done, self.info()

    def _step_plan(self, cols: int) -> dict:
        """step()'s wg_step_ranges arguments for this env's own output tensors, cached per (generation, batch struct,
        action columns): one wg_range per walker range (uniform: offset batch views; ragged: plan slices), the
        outputs, the action element offset of each range, its stream, and the fork / join events."""
        key = (self._generation, id(self.batch.struct), cols)
        cached = getattr(self, "_plan_cache", None)
        if cached is not None and cached["key"] == key:
            return cached
        lanes = self._step_lanes() if cols >= 0 else 1
        self.reserve_streams(lanes)
        b = self.batch
        keep = []                                  # the ctypes structs the ranges point at
        rng = (_lib.WgRange * lanes)()

        def out(w0, w1):
            o = self._outputs(self.obs[w0:w1], self.reward[w0:w1], self.done[w0:w1], self.centroid[w0:w1],
                              self.energy[w0:w1], pad_clean=True,
                              steps=None if self.steps_out is None else self.steps_out[w0:w1],
                              **self._extra_out(w0, w1))
            keep.append(o)
            return C.pointer(o)
        if lanes == 1 or b.ragged:
            nb = b.plan_blocks
            bounds = [nb * i // lanes for i in range(lanes)] + [nb]
            o = out(0, self.N)
            for i in range(lanes):
                rng[i].batch, rng[i].outputs, rng[i].action_offset = C.pointer(b.struct), o, 0
                rng[i].plan = None if b.plan is None else b.plan.data_ptr() + 4 * bounds[i]
                rng[i].plan_blocks = bounds[i + 1] - bounds[i] if b.plan is not None else 0
        else:
            bounds = [0] + [((self.N * i // lanes) + 63) // 64 * 64 for i in range(1, lanes)] + [self.N]
            for i in range(lanes):
                w0, w1 = bounds[i], bounds[i + 1]
                sub = b.sub_struct(w0, w1)
                keep.append(sub)
                rng[i].batch, rng[i].outputs = C.pointer(sub), out(w0, w1)
                rng[i].action_offset, rng[i].plan, rng[i].plan_blocks = w0 * max(cols, 0), None, 0
        side = self._side[:lanes - 1]
        for i, st in enumerate(side):
            rng[i + 1].stream = st.cuda_stream
        events = [torch.cuda.Event() for _ in range(lanes)]
        for ev in events:
            ev.record()                            # materialise the hipEvent handle
        self._pref = C.byref(self._pstruct)
        self._plan_cache = {"key": key, "fn": _lib.load().wg_step_ranges, "ranges": rng, "n": lanes, "side": side,
                            "keep": keep, "events_obj": events,
                            "events": (C.c_void_p * lanes)(*[ev.cuda_event for ev in events])}
        return self._plan_cache

    def rollout(self, actions, obs_out=None, reward_out=None, done_out=None, lanes: Optional[int] = None,
                resident: bool = True):
        """T steps in one C call, no host sync; outputs for every step.  resident (default): wg_rollout, one launch
        for all T steps where the batch allows it (uniform M | 64, no pair forces), each walker's state kept in
        registers between steps; False: wg_step, one launch per step.  Bit-identical either way."""
        if not isinstance(actions, torch.Tensor):
            actions = torch.as_tensor(np.asarray(actions, dtype=np.float32))
        actions = actions.to(self.device, torch.float32).contiguous()
        if actions.dim() != 3 or actions.shape[1] != self.N:
            raise ValueError("actions must be [T, N, A]")
        T, _, cols = actions.shape
        dv = self.device
        self._steps_at = -1   # the step counters move without the steps output: info() gathers them afterwards
        # (the per-step outputs went to the rollout's buffers: the env's own centroid / energy / extras are not current)
        self._stale = frozenset({"centroid_position", "total_energy", "momentum", "nonfinite"})
        # zero-filled: a ragged batch's short rows then need only their own values written each step
        clean = obs_out is None
        obs_out = torch.zeros((T, self.N, self.obs_dim), dtype=torch.float32, device=dv) if obs_out is None else obs_out
        reward_out = torch.empty((T, self.N), dtype=torch.float32, device=dv) if reward_out is None else reward_out
        done_out = torch.empty((T, self.N), dtype=torch.uint8, device=dv) if done_out is None else done_out
        require_tensor(obs_out, "obs_out", dv, torch.float32, (T, self.N, self.obs_dim))
        require_tensor(reward_out, "reward_out", dv, torch.float32, (T, self.N))
        require_tensor(done_out, "done_out", dv, torch.uint8, (T, self.N))
        # one resident launch holds its walkers for all T steps: no per-step launch tail for a second range to fill
        # (profiles/r02_ab_resident_occupancy.json: 38.2 us/step with one range, 39.6 with two)
        # (only where the resident kernel actually runs: otherwise the default walker ranges keep their overlap)
        lanes = self._lanes(1 if (resident and lanes is None and self.resident_ok()) else lanes) if T > 0 else 1
        entry = "wg_rollout" if resident else "wg_step"
        o = self._outputs(obs_out, reward_out, done_out, None, None, obs_step=self.N * self.obs_dim,
                          out_step=self.N, pad_clean=clean)
        if lanes > 1:
            self._run_lanes(actions, T, o, lanes, entry=entry)
            return obs_out, reward_out, done_out
        _lib.check(getattr(_lib.load(), entry)(
            C.byref(self.batch.struct), C.byref(self._pstruct), C.c_void_p(actions.data_ptr()), cols, cols,
            self.N * cols, C.byref(o), T,
            None if self.batch.plan is None else C.c_void_p(self.batch.plan.data_ptr()),
            self.batch.plan_blocks, self._stream()), entry)
        return obs_out, reward_out, done_out

    def run(self, actions, n_steps: int, info: bool = True, lanes: Optional[int] = None, resident: bool = False,
            record: Optional[dict] = None, _only: Optional[int] = None):
        """Throughput path: n_steps env steps in one C call; step s acts with actions[s % T]
        ([T, N, A] device tensor; T == n_steps or 1) and overwrites obs/reward/done(/info) each step.  resident:
        wg_rollout (one launch for all steps where the batch allows it) instead of one launch per step.

        record: every step's reward / done (and with info, energy / centroid) into caller buffers instead of the
        env's one-step outputs — {'reward': [n_steps, N] f32, 'done': [n_steps, N] bool or u8, optionally 'energy'
        [n_steps, N] f32 and 'centroid' [n_steps, N, 3] f32} — while obs keeps the last step's rows (env.obs): the
        rollout SURVEY §8(e) gathers at its end.  The same bytes as a plain run, written at per-step offsets.  After a
        record run env.reward / done / centroid / energy and the info extras are not this run's (they went to the
        record buffers, or were not computed): info() leaves those keys out until the next step() / observe() / run()
        without record."""
        self.prepare_run(actions, n_steps, info=info, lanes=lanes, resident=resident, record=record, _only=_only)()

    def prepare_run(self, actions, n_steps: int, info: bool = True, lanes: Optional[int] = None,
                    resident: bool = False, record: Optional[dict] = None,
                    _only: Optional[int] = None) -> "PreparedRun":
        """run()'s argument checks, walker ranges and C structs, built once: the returned PreparedRun issues the same
        n_steps steps with ONE C call each time it is called (on the stream that was current here), so the host time
        between a caller's clock start and the first launch is one ctypes call (bench.py builds it before its timed
        region: ~35 us of Python before the first launch otherwise).  It holds raw pointers to `actions`,
        the record buffers and the env's tensors: set_params / a reallocation of the outputs make it raise.
        (_only = i, graph() only: walker range i alone, on the calling stream.)"""
        require_tensor(actions, "actions", self.device, torch.float32)
        if actions.dim() != 3:
            raise ValueError("actions must be a contiguous [n_steps or 1, N, A] device tensor")
        T, n, cols = actions.shape
        if n != self.N or T not in (1, n_steps):
            raise ValueError("actions must be a contiguous [n_steps or 1, N, A] device tensor")
        lanes = self._lanes(1 if (resident and lanes is None and self.resident_ok()) else lanes)
        entry = "wg_rollout" if resident else "wg_step"
        so = self.steps_out if info else None
        rew, done, cen, en, out_step = self.reward, self.done, self.centroid, self.energy, 0
        stale = set()
        if record is not None:
            S = int(n_steps)
            if S < 1:
                raise ValueError("run(record=...) needs n_steps >= 1")
            stale = {"centroid_position", "total_energy", "momentum", "nonfinite"}
            rew, done = record["reward"], record["done"]
            require_tensor(rew, "record['reward']", self.device, torch.float32, (S, self.N))
            if not isinstance(done, torch.Tensor) or done.dtype not in (torch.bool, torch.uint8):
                raise ValueError("record['done'] must be a bool or uint8 tensor")
            require_tensor(done, "record['done']", self.device, done.dtype, (S, self.N))
            cen, en = record.get("centroid"), record.get("energy")
            if cen is not None:
                require_tensor(cen, "record['centroid']", self.device, torch.float32, (S, self.N, 3))
            if en is not None:
                require_tensor(en, "record['energy']", self.device, torch.float32, (S, self.N))
            rew, done = rew[0], done[0]
            cen, en = (None if cen is None else cen[0]), (None if en is None else en[0])
            so, out_step = None, self.N   # (the steps output would need [n_steps, N] too: info() gathers them)
        if not info:
            cen = en = None
            stale |= {"centroid_position", "total_energy", "momentum", "nonfinite"}
        # the opt-in info extras follow the last step only when the outputs are overwritten each step (no record)
        o = self._outputs(self.obs, rew, done, cen, en, pad_clean=True, steps=so, out_step=out_step,
                          **(self._extra_out() if (info and record is None) else {}))
        # every tensor whose raw pointer sits in `o`, held by the PreparedRun (a caller that drops its record
        # buffers and calls the PreparedRun again must not have the kernel write into freed memory)
        pins = [self.obs, so, actions, *(() if record is None else record.values()), *self._extra_out().values()]
        steps_valid = so is not None
        n_steps = int(n_steps)
        if lanes > 1:
            capturing = torch.cuda.is_current_stream_capturing()
            if entry == "wg_step" and not capturing and _only is None and \
                    os.environ.get("WG_RANGE_ISSUE", "inter") != "seq":
                fn, args, keep = self._run_ranges_args(actions, n_steps, o, lanes)
                if n_steps > 0:
                    for st in self._side[:lanes - 1]:
                        actions.record_stream(st)   # the allocator must not recycle it before the side streams are done
                return PreparedRun(self, "wg_run_ranges", fn, args, keep + pins, steps_valid, stale)
            # (range-by-range issue, a resident rollout over several ranges, or a graph capture: one C call per range)
            return PreparedRun(self, entry, None, (actions, n_steps, o, lanes, entry, _only), [o] + pins, steps_valid,
                               stale, thunk=self._run_lanes)
        # (a resident launch writes the steps output only where the resident kernel runs: uniform batches, which
        # have no steps_out)
        args = (C.byref(self.batch.struct), C.byref(self._pstruct), actions.data_ptr(), cols, cols,
                0 if T == 1 else self.N * cols, C.byref(o), n_steps,
                None if self.batch.plan is None else self.batch.plan.data_ptr(), self.batch.plan_blocks,
                torch.cuda.current_stream(self.device).cuda_stream)
        return PreparedRun(self, entry, getattr(_lib.load(), entry), args, [o] + pins, steps_valid, stale)

    def time_launches(self, actions, n_steps: int, info: bool = True) -> float:
        """Measurement aid (bench.py's roofline): run(actions, n_steps, lanes=1)'s steps — one full-batch launch per
        step, the same results — with each step kernel's own start and end stamped on events of its own (wg_time_step,
        hipExtLaunchKernel: the dispatch's timestamps, as a kernel trace reports them, without the gaps between
        back-to-back launches).  Waits for the calling stream; returns the mean kernel duration in ms."""
        prep = self.prepare_run(actions, n_steps, info=info, lanes=1)
        ms = C.c_float(0.0)
        _lib.check(_lib.load().wg_time_step(*prep._args, C.byref(ms)), "wg_time_step")
        self._steps_at = self.batch.version if prep._steps_valid else -1   # (as PreparedRun.__call__)
        self._stale = prep._stale
        return float(ms.value)

    def _lanes(self, lanes: Optional[int]) -> int:
        """Walker ranges run() steps on separate streams (ragged batches: ranges of plan blocks).  Default 2 for
        batches of >= 2^19 masses: measured on the canonical 65,536-walker bench (2^20 masses), 36.5 us/step
        with 2 ranges against 42.9 with 1 and 49.0 with 4; on 65,536 Balance-v0 walkers (2^18 masses, a 13 us
        launch) 2 ranges lose slightly, 13.7 against 13.3 (scripts/lanes_ab.py; bit-identical results).  Pair
        forces (O(M^2) per walker) make launches long at fewer masses: 4,096 chain walkers of 100 masses (2^18.6),
        175 us/step with 2 ranges against 210 with 1 (profiles/r02_ab_pair_markstein_chain.json), so those
        batches take 2 ranges from 2^17 masses.  WG_LANES overrides."""
        if lanes is None:
            env = os.environ.get("WG_LANES")
            heavy = int(self.params.pair_mode) != 0
            lanes = int(env) if env else (2 if self.batch.P >= (1 << (17 if heavy else 19)) else 1)
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        if self.batch.ragged:
            return max(1, min(lanes, self.batch.plan_blocks // 64))
        return 1 if self.N < 64 * lanes else lanes

    def _step_lanes(self) -> int:
        """Walker ranges of step(): 1 unless WG_STEP_LANES says otherwise.  step() joins its ranges at the end of
        every call, so a second range cannot fill the first one's launch tail with its next step (what pays in
        run()), and the fork / join events cost host time on every call: measured on the canonical 65,536-walker
        batch, a step() loop ran 47.7 us per step with 1 range against 58.5 with 2 (host 7.8 against 25.1 us per
        call; scripts/step_overhead.py, profiles/r03g_step_overhead_canonical.json)."""
        env = os.environ.get("WG_STEP_LANES")
        return self._lanes(int(env)) if env else 1

    def reserve_streams(self, lanes: int) -> None:
        """Side streams for `lanes` walker ranges (lanes - 1 of them; existing ones are kept, so their hardware
        queues stay bound).  Call before creating other streams (an RCCL process group) to keep the ranges on
        queues of their own."""
        while len(self._side) < lanes - 1:
            self._side.append(torch.cuda.Stream(device=self.device))

    def _range_batches(self, lanes: int, bounds) -> list:
        """The per-range WgBatch views of a uniform batch, cached per batch struct (rebuilt whenever the batch's
        arrays are: enable_radius) and walker ranges; the cache holds the struct, so its identity is not reused."""
        key, st = (self._generation, tuple(bounds)), self.batch.struct
        cached = getattr(self, "_range_cache", None)
        if cached is None or cached[0] != key or cached[1] is not st:
            cached = self._range_cache = (key, st, [self.batch.sub_struct(bounds[i], bounds[i + 1]) for i in range(lanes)])
        return cached[2]

    def _range_bounds(self, lanes: int) -> list:
        """Walker ranges of run(): plan-block bounds (ragged: the same batch, a slice of its block -> walker plan) or
        walker bounds on multiples of 64 (uniform)."""
        if self.batch.ragged:
            nb = self.batch.plan_blocks
            return [nb * i // lanes for i in range(lanes)] + [nb]
        return [0] + [((self.N * i // lanes) + 63) // 64 * 64 for i in range(1, lanes)] + [self.N]

    def _run_ranges_args(self, actions, n_steps: int, o_full, lanes: int):
        """wg_run_ranges' arguments for n_steps of `lanes` walker ranges on the calling stream and the side streams:
        step s of every range is issued before step s + 1 of any (WG_RANGE_ISSUE=seq keeps range-by-range issue, one
        wg_step call each: the last range then starts only after the host has issued every launch of the ranges
        before it; scripts/issue_ab.sh).  Returns (function, arguments, the ctypes objects they point at)."""
        T, n, cols = actions.shape
        cur = torch.cuda.current_stream(self.device)
        self.reserve_streams(lanes)
        ragged = self.batch.ragged
        bounds = self._range_bounds(lanes)
        rng, keep = (_lib.WgRange * lanes)(), []
        subs = None if ragged else self._range_batches(lanes, bounds)
        for i in range(lanes):
            w0, w1 = bounds[i], bounds[i + 1]
            if ragged:
                o, rng[i].batch, rng[i].action_offset = o_full, C.pointer(self.batch.struct), 0
                rng[i].plan, rng[i].plan_blocks = self.batch.plan.data_ptr() + 4 * w0, w1 - w0
            else:
                o, rng[i].batch, rng[i].action_offset = self._range_outputs(o_full, w0), C.pointer(subs[i]), w0 * cols
                rng[i].plan, rng[i].plan_blocks = None, 0
            keep.append(o)
            rng[i].outputs = C.pointer(o)
            rng[i].stream = (cur if i == 0 else self._side[i - 1]).cuda_stream
        keep += [rng, o_full, actions, subs]
        args = (rng, lanes, C.byref(self._pstruct), actions.data_ptr(), cols, cols, 0 if T == 1 else self.N * cols,
                n_steps, self._range_events(lanes))
        return _lib.load().wg_run_ranges, args, keep

    def _run_lanes(self, actions, n_steps: int, o_full, lanes: int, entry: str = "wg_step", only: Optional[int] = None):
        """n_steps with the walkers split into `lanes` contiguous ranges, each stepped by its own stream, one C call
        per range (the range-by-range form; prepare_run issues the ranges step by step through wg_run_ranges): the
        ranges are independent, so one range's step t + 1 fills the GPU while another's step t drains (the
        launch tail).  Every walker still takes every step, one launch per step per range; the calling
        stream waits for all ranges before returning (stream-ordered, no host sync).  o_full: the whole batch's
        WgOutputs (a uniform range's are its pointers advanced to the range's first walker).  only = i: range i
        alone, on the calling stream (graph() captures one graph per range)."""
        T, n, cols = actions.shape
        cur = torch.cuda.current_stream(self.device)
        self.reserve_streams(lanes)
        L = _lib.load()
        ragged = self.batch.ragged
        bounds = self._range_bounds(lanes)
        capturing = torch.cuda.is_current_stream_capturing()
        start = torch.cuda.Event()
        if only is None:
            start.record(cur)
        done = []
        for i in (range(lanes) if only is None else [only]):
            w0, w1 = bounds[i], bounds[i + 1]
            st = cur if (i == 0 or only is not None) else self._side[i - 1]
            if st is not cur:
                st.wait_event(start)
            if ragged:
                sub, o, act = self.batch.struct, o_full, C.c_void_p(actions.data_ptr())
                plan, nblk = C.c_void_p(self.batch.plan.data_ptr() + 4 * w0), w1 - w0
            else:
                sub, o = self.batch.sub_struct(w0, w1), self._range_outputs(o_full, w0)
                act, plan, nblk = C.c_void_p(actions.data_ptr() + 4 * w0 * cols), None, 0
            _lib.check(getattr(L, entry)(C.byref(sub), C.byref(self._pstruct), act, cols, cols,
                                         0 if T == 1 else self.N * cols, C.byref(o), n_steps, plan, nblk,
                                         C.c_void_p(st.cuda_stream)), entry)
            if st is not cur:
                if not capturing:
                    actions.record_stream(st)   # the allocator must not recycle it before the side stream is done
                ev = torch.cuda.Event()
                ev.record(st)
                done.append(ev)
        for ev in done:
            cur.wait_event(ev)

    def _range_events(self, lanes: int):
        """wg_run_ranges' fork / join events (hipEvent handles of torch events, created once per env and reused: each
        call records and waits on them stream-ordered)."""
        ev = getattr(self, "_run_events", None)
        if ev is None or len(ev[0]) < lanes:
            objs = [torch.cuda.Event() for _ in range(lanes)]
            for e in objs:
                e.record()                       # materialise the hipEvent handle
            ev = self._run_events = (objs, (C.c_void_p * lanes)(*[e.cuda_event for e in objs]))
        return ev[1]

    def policy_loop(self, policy, n_steps: int, lanes: Optional[int] = None, graph: bool = False) -> None:
        """A closed loop with a per-walker policy, the walker ranges pipelined: at every step, each range computes its
        actions from ITS OWN current observation rows, action = policy(obs[w0:w1], t), and launches its step right
        after, on its own stream; the ranges never wait for one another.  So one range's step t + 1 fills the other's
        launch tail, as in the open-loop run(), while every action still depends on the observation it follows.
        step() in a loop cannot do that: it returns the whole batch's obs, so each step ends at a full barrier and
        each launch drains on its own (the drain is what separates one launch from two overlapped ranges).

        policy(obs_rows [n_r, D] view, t) -> actions [n_r, A_cols] float32, contiguous, on the current (range)
        stream.  It must be row-wise — walker w's action a function of walker w's observation only — which is what
        makes the ranges independent; then the results are bit-identical to `for t: env.step(policy(env.obs, t))`.
        graph=True captures the n_steps x ranges loop (policy kernels included) as one HIP graph and replays it once
        (no per-step host cost; the policy must be capturable).  After the call obs / reward / done / info hold the last
        step's outputs.

        Ragged batches (stored in wave-tile order, wg_batch.row) run ranges of plan blocks.  The wave tiles are packed
        within windows of consecutive caller walkers (layout.wave_tile_order), so a range that ends at a block whose
        stored prefix is exactly the caller rows before it covers a contiguous slice of caller rows: the ranges are
        split at the such block nearest to an even split (_caller_bounds), and each range reads its obs rows as a
        slice and hands the kernel its actions as given.  Where no such block is near, a range's walkers are a
        scattered set of caller rows: it gathers its rows of obs (index_select), applies the policy and scatters the
        actions into its rows of one [N, A] action buffer (index_copy_), which its step reads by caller row.  Either
        way the ranges' rows are disjoint, so they never wait for one another.

        Host cost per range and step (what bounds a small batch's loop): the policy's own launches, a shape / dtype
        check against the first step's actions, and one C call; the stream is switched only when there are several
        ranges (one range runs on the calling stream as it is)."""
        b = self.batch
        lanes = self._lanes(lanes)
        self.reserve_streams(lanes)
        L = _lib.load()
        pref, dev, f32 = C.byref(self._pstruct), self.device, torch.float32
        args = []   # per range: (obs rows or None, row index or None, n_r, batch ref, outputs ref, plan ptr, blocks)
        keep = []   # the ctypes structs the refs point at
        aoff = []   # per range: the caller row its actions start at (the kernel indexes a ragged batch's actions by
        #             caller row, so a slice's action pointer is moved back by that many rows)
        if b.ragged:
            bb, contiguous = self._caller_bounds(lanes)
            o = self._outputs(self.obs, self.reward, self.done, self.centroid, self.energy, pad_clean=True,
                              steps=self.steps_out, **self._extra_out())
            keep.append(o)
            for i in range(lanes):
                s0, s1 = int(b.plan_host[bb[i]]), int(b.plan_host[bb[i + 1]])
                if contiguous[i]:   # caller rows s0 .. s1 - 1: a row slice
                    obs_r, idx = self.obs[s0:s1], None
                else:               # the caller rows of stored walkers s0 .. s1 - 1, scattered
                    obs_r, idx = None, b._perm["row"][s0:s1]
                aoff.append(s0)
                args.append((obs_r, idx, s1 - s0, C.byref(b.struct), C.byref(o),
                             C.c_void_p(b.plan.data_ptr() + 4 * bb[i]), bb[i + 1] - bb[i]))
        else:
            bounds = [0] + [((self.N * i // lanes) + 63) // 64 * 64 for i in range(1, lanes)] + [self.N]
            for i in range(lanes):
                w0, w1 = bounds[i], bounds[i + 1]
                sub = b.sub_struct(w0, w1)
                o = self._outputs(self.obs[w0:w1], self.reward[w0:w1], self.done[w0:w1], self.centroid[w0:w1],
                                  self.energy[w0:w1], pad_clean=True, **self._extra_out(w0, w1))
                keep += [sub, o]
                args.append((self.obs[w0:w1], None, w1 - w0, C.byref(sub), C.byref(o), None, 0))
                aoff.append(0)   # (a sub-batch indexes its actions from its own first walker)

        def check(a, n_r):
            require_tensor(a, "policy actions", dev, f32)
            if a.dim() != 2 or a.shape[0] != n_r:
                raise ValueError(f"policy returned {tuple(a.shape)}, expected [{n_r}, A]")

        def body(cur, only=None):
            # only = r: range r's loop alone, on `cur` (graph mode captures one graph per range)
            multi = lanes > 1 and only is None
            streams = [cur] + self._side[:lanes - 1] if only is None else [cur]
            if multi:
                start = torch.cuda.Event()
                start.record(cur)
                for st in streams[1:]:
                    st.wait_event(start)
            step = L.wg_step
            sts = [(st, st.cuda_stream) for st in streams]
            rng = list(enumerate(args)) if only is None else [(only, args[only])]
            shapes = [None] * lanes
            dix = dev.index
            # scattered ragged ranges: the [N, A] action buffer they scatter into.  Its columns are known only from the
            # first policy call, so it is allocated then, on `cur` (uninitialised: every range writes its own rows
            # before its step reads them), and an event recorded on `cur` right after the allocation orders every
            # stream that touches it after whatever `cur` ran in that memory before (the caching allocator reuses a
            # block freed on `cur` without waiting for other streams); the ranges' streams join `cur` at the end, so
            # its release on `cur` is ordered after their last reads
            abuf, abuf_ev, abuf_ok = None, None, set()
            try:
                for t in range(int(n_steps)):
                    for (r, (obs_r, idx, n_r, b_ref, o_ref, plan, nblk)), (st, st_ptr) in zip(rng, sts):
                        if multi:
                            torch.cuda.set_stream(st)
                        a = policy(obs_r if idx is None else self.obs.index_select(0, idx), t)
                        # the full check at a range's first step, then the same shape, dtype, device and layout
                        if shapes[r] is None:
                            check(a, n_r)
                            if r > 0 and shapes[0] is not None and a.shape[1] != shapes[0][1]:
                                raise ValueError("policy actions: every walker range must return the same columns")
                            shapes[r] = a.shape
                        elif not (a.shape == shapes[r] and a.dtype == f32 and a.get_device() == dix and
                                  a.is_contiguous()):
                            check(a, n_r)
                            raise ValueError(f"policy actions changed shape: {tuple(a.shape)} after "
                                             f"{tuple(shapes[r])}")
                        cols = a.shape[1]
                        if idx is not None:   # a scattered ragged range: its caller rows of the action buffer
                            if abuf is None:
                                with torch.cuda.stream(cur):
                                    abuf = torch.empty((self.N, cols), dtype=f32, device=dev)
                                abuf_ok.add(cur.cuda_stream)
                                if multi:   # (one stream, e.g. a captured range: nothing to order)
                                    abuf_ev = torch.cuda.Event()
                                    abuf_ev.record(cur)
                            if abuf_ev is not None and st_ptr not in abuf_ok:
                                st.wait_event(abuf_ev)
                                abuf_ok.add(st_ptr)
                            abuf.index_copy_(0, idx, a)
                            a_ptr = abuf.data_ptr()
                        else:                 # (rows aoff[r] .. of the caller's order: the pointer moved back)
                            a_ptr = a.data_ptr() - 4 * aoff[r] * cols
                        rc = step(b_ref, pref, a_ptr, cols, cols, 0, o_ref, 1, plan, nblk, st_ptr)
                        if rc:
                            _lib.check(rc, "wg_step")
            finally:
                if multi:
                    torch.cuda.set_stream(cur)
            for st in streams[1:]:
                ev = torch.cuda.Event()
                ev.record(st)
                cur.wait_event(ev)

        self._steps_at = -1
        self._stale = frozenset()
        cur = torch.cuda.current_stream(self.device)
        if not graph:
            body(cur)
            return
        # one graph per walker range, each replayed on a stream of its own: the ranges share nothing, and two graphs
        # on two streams overlap as the eager ranges do (one graph with the ranges as parallel branches replayed them
        # one after the other: 48.1 against 38.1 us per canonical step, round 4)
        parts = []
        for r in range(lanes):
            g = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream(device=self.device)
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                with torch.cuda.graph(g, stream=st):
                    body(st, only=r)
            cur.wait_stream(st)
            parts.append((g, st))
        self._policy_graph = _RangeGraphs(parts, cur)   # (kept until the next call: the replay may still be running)
        self._policy_graph.replay()

    def _caller_bounds(self, lanes: int):
        """Plan-block bounds of `lanes` ragged walker ranges, each split moved to the nearest block whose stored prefix
        holds exactly the caller rows before it (within an eighth of a range), and per range whether its walkers are a
        contiguous slice of caller rows."""
        b = self.batch
        nb, plan = b.plan_blocks, b.plan_host
        if b.row is None:
            ok = np.ones(nb + 1, bool)   # identity order: every block boundary
        else:
            rowmax = np.maximum.accumulate(b.host.row)
            ok = np.zeros(nb + 1, bool)
            ok[0] = ok[nb] = True
            s = plan[1:nb].astype(np.int64)
            ok[1:nb] = rowmax[s - 1] == s - 1
        good = np.flatnonzero(ok)
        bb = [0]
        for i in range(1, lanes):
            t = nb * i // lanes
            c = int(good[np.argmin(np.abs(good - t))])
            bb.append(c if abs(c - t) <= max(1, nb // (8 * lanes)) and bb[-1] < c < nb else t)
        bb.append(nb)
        contiguous = [bool(ok[bb[i]] and ok[bb[i + 1]]) for i in range(lanes)]
        return bb, contiguous

    def graph(self, actions, n_steps: int, info: bool = True, lanes: Optional[int] = None):
        """Capture run(actions, n_steps) into a HIP graph (torch.cuda.CUDAGraph over the ROCm runtime) and
        return it as a WalkerGraph; replay() then advances the batch n_steps with one host call: one graph per walker
        range, each replayed on its own stream, forked from and joined back to the calling stream (_RangeGraphs).  `actions` is kept alive by the WalkerGraph (and may be
        refilled in place); the graph reads the batch and output tensors this env owns and the parameters as
        captured, so set_params() (or any reallocation of the outputs) makes replay() raise."""
        lanes = self._lanes(lanes)
        cur = torch.cuda.current_stream(self.device)
        steps_at, stale = self._steps_at, self._stale   # capture runs nothing: the outputs' validity is unchanged
        parts = []
        for r in range(lanes):   # one graph per walker range, each replayed on a stream of its own (_RangeGraphs)
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream(device=self.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):           # capture off the default stream, as torch requires
                with torch.cuda.graph(g, stream=side):
                    self.run(actions, n_steps, info=info, lanes=lanes, _only=r if lanes > 1 else None)
            cur.wait_stream(side)
            parts.append((g, side))
        self._steps_at, self._stale = steps_at, stale
        return WalkerGraph(self, _RangeGraphs(parts, cur), actions, info=info)

    def observe(self):
        o = self._outputs(self.obs, self.reward, self.done, self.centroid, self.energy, steps=self.steps_out,
                          **self._extra_out())
        _lib.check(_lib.load().wg_observe(
            C.byref(self.batch.struct), C.byref(self._pstruct), C.byref(o),
            None if self.batch.plan is None else C.c_void_p(self.batch.plan.data_ptr()),
            self.batch.plan_blocks, self._stream()), "wg_observe")
        self._steps_at = self.batch.version
        self._stale = frozenset()
        return self.obs, self.reward, self.done, self.info()

    def reset(self, noise=None, mask=None):
        """PhysicsEnv.reset: v += N(0, sigma) noise on x, y (and z if in3d); steps = 0; returns obs.
        ``noise`` [P, 3] overrides the device generator (use it for reproducible parity runs)."""
        if noise is None and self.sigma > 0:
            noise = torch.randn((self.batch.P, 3), generator=self._gen, device=self.device) * self.sigma
        if noise is not None:   # caller's mass order -> the stored order
            noise = self.batch.to_stored("mass", torch.as_tensor(noise, dtype=torch.float32).to(self.device)
                                         .reshape(self.batch.P, 3)).contiguous()
        if mask is not None:
            mask = self.batch.to_stored("walker", torch.as_tensor(mask).to(self.device, torch.uint8)).contiguous()
        _lib.check(_lib.load().wg_reset(
            C.byref(self.batch.struct), C.byref(self._pstruct),
            None if noise is None else C.c_void_p(noise.data_ptr()),
            None if mask is None else C.c_void_p(mask.data_ptr()), self._stream()), "wg_reset")
        return self.observe()[0]

    def seed(self, seed: Optional[int] = None) -> Sequence[int]:
        if seed is not None:
            self._gen.manual_seed(int(seed))
        return [seed] if seed is not None else []

    def info(self) -> dict:
        if self.steps_out is not None and self._steps_at == self.batch.version:
            steps = self.steps_out                 # written by the last step / observe in caller order
        else:
            steps = self.batch.caller("steps")     # a gather (after a rollout, a reset mask, or loaded state)
        info = {"steps": steps, "centroid_position": self.centroid, "total_energy": self.energy}
        if self._extras:
            info["momentum"] = self.momentum      # Point.momentum (gym/engine.py:160-166) of each walker
            info["nonfinite"] = self.nonfinite    # True: the walker's pos / vel / acc hold an inf or NaN
        for k in self._stale:                     # not written by the last run() (record buffers, info=False)
            info.pop(k, None)
        return info

    # state accessors in the caller's order.  An unpermuted batch returns live views into its tensors; a ragged batch
    # (stored in wave-tile / size order) returns gathered COPIES, so in-place writes into them do not reach the batch:
    # assign instead (env.pos = t, env.vel[...] edits then env.vel = edited), which scatters into the stored order.
    def _set_state(self, name: str, value) -> None:
        self.batch.version += 1
        dst = getattr(self.batch, name)
        t = torch.as_tensor(value, dtype=dst.dtype).to(self.device).reshape(dst.shape)
        dst.copy_(self.batch.to_stored(self.batch.KIND[name], t))

    @property
    def pos(self):
        return self.batch.caller("pos")

    @pos.setter
    def pos(self, value):
        self._set_state("pos", value)

    @property
    def vel(self):
        return self.batch.caller("vel")

    @vel.setter
    def vel(self, value):
        self._set_state("vel", value)

    @property
    def acc(self):
        return self.batch.caller("acc")

    @acc.setter
    def acc(self, value):
        self._set_state("acc", value)

    @property
    def muscle_x(self):
        return self.batch.caller("muscle_x")

    @muscle_x.setter
    def muscle_x(self, value):
        self._set_state("muscle_x", value)

    @property
    def contact(self):
        return self.batch.caller("contact")

    @property
    def steps(self):
        return self.batch.caller("steps")

    def get_action_space(self) -> dict:
        return {"shape": (self.batch.A,), "type": "continuous", "low": -1.0, "high": 1.0}

    def get_observation_space(self) -> dict:
        return {"shape": (self.obs_dim,), "type": "continuous", "low": -np.inf, "high": np.inf}

    def launch_geometry(self) -> dict:
        return self.batch.launch_geometry()
