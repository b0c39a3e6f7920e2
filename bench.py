#!/usr/bin/env python3
"""Headline benchmark: env-steps/sec of the batched walker stepper (BASELINE.json `metric`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--walkers 65536] [--workload canonical]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N` without a torch.distributed world starts the N rank processes itself (torch.distributed.run, before
any GPU call) and exits with their status; inside a world whose size differs from --gpus it exits with 2.

A step = one env step (act -> springs -> env forces -> run1 -> obs/reward/done/info) over the rank's batch,
with obs/reward/done/info materialised every step.  The batch is split into walker ranges stepped on separate
HIP streams (BatchedPhysicsEnv.run lanes: 2 for batches of >= 2^19 masses), one launch per range per step:
every walker takes every step, and one range's next step fills the GPU while the other's drains.  Inputs
(state, topology and a distinct U(-1,1) action tensor for every timed step) are resident in HBM before timing.
Weak scaling: each rank owns its own `--walkers` walkers (no data-path collective).  Inside a torch.distributed world
RCCL's communicator is created before the env's warm-up and checked (`comm`: its size by an all_reduce of ones, every
rank's PCI address distinct), the job time is max(t1) - min(t0) over ranks on the node's shared clock, and
the rollout-end gather (RCCL all_gather_into_tensor of the final observations and the per-step reward / done records)
runs after the barrier that closes the K timed steps (`--gather serial`, the default): `value` is the K steps,
`value_incl_gather` the steps and the gather, and `gather.content_check` compares every rank's checksums of what it
sent with its shard of the gathered tensors (a failed check exits 3).  `--gather pipelined` gathers the previous
rollout's observations while this one steps, inside the timed region (slower on one MI355X).
After the K steps `sustained` times 1,000 steps and a ~2 s run of the same walker ranges (the long-run clock).
Rank 0 prints ONE JSON line.  Workloads: canonical (M=16, K=40, A=8; config 3/4),
balance (Balance-v0; config 2 at --walkers 4096), ragged (M ~ U{4..32}; config 5), chain (performance_demo's
chain of --chain-points masses with per-walker Point.gravity; §8(f) 3).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node) at 65 536 walkers; 1/2/4/8 MI355X scaling"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# vector (non-matrix) VALU peaks: FP32 157.3 TFLOP/s is MI355X_MICROARCH.md's (v_pk_fma_f32); the guide lists no FP64
# figure, so FP64 is AMD's MI355X datasheet vector FP64, 78.6 TFLOP/s (= the FP32 rate without packing: one v_fma_f64
# per lane per 2 cycles); scripts/valu_peak.hip measures both on the box (profiles/r03_valu_peak.json)
FP64_PEAK_TFS = 78.6
FP32_PEAK_TFS = 157.3
# algorithmic FLOP per unordered pair of the reference's pair loops:
#   chain (gym/engine.py:128-137 + anti_forced :69-76): 3 norms x 2 float64 adds, r**2, two products and the
#     quotient of f, and per end 3 products, 3 quotients by r, 3 by m, 3 adds: 34 FP64
#   perfdemo (gym/optimized_engine.py:177-193, gravity_vec): float32 norm (3 products, sqrt) and powf, the quotient
#     of f, 3 products and 3 quotients of the force, and per end 3 quotients by m and 3 adds: 24 FP32
#     (+ the norm's 2 float64 adds and the numerator's 2 float64 products)
PAIR_FLOP = {"chain": (34, "fp64-valu", FP64_PEAK_TFS), "perfdemo": (24, "fp32-valu", FP32_PEAK_TFS)}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)   # time 1,000 steps after 50
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--walkers", type=int, default=65536, help="walkers per GPU")
    ap.add_argument("--workload", default="canonical",
                    choices=["canonical", "balance", "ragged", "chain", "perfdemo", "lattice25"])
    ap.add_argument("--chain-points", type=int, default=100, help="masses per chain walker (--workload chain)")
    ap.add_argument("--lanes", type=int, default=None, help="walker ranges on separate streams (default: auto)")
    ap.add_argument("--resident", action="store_true", help="also time the K steps as ONE wg_rollout launch (state in "
                    "registers across steps; open-loop actions) and report it beside the line (not the headline)")
    ap.add_argument("--graph", action="store_true", help="time a HIP-graph replay of the K steps (and the direct "
                                                         "calls beside it)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline samples")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--gather-to", choices=["root", "all"], default="all",
                    help="rollout-end collective: all = all_gather_into_tensor into every rank (RCCL's ring "
                         "collective); root = dist.gather to rank 0 (the learner; peer-to-peer sends)")
    ap.add_argument("--gather", choices=["serial", "pipelined"], default="serial",
                    help="rollout-end observation gather inside the timed region: serial (default: this rollout's "
                         "final observations, after its last step) or pipelined (the previous rollout's, gathered "
                         "while this rollout steps; measured slower on one MI355X: RCCL's kernels stall the steps)")
    ap.add_argument("--no-control", action="store_true", help="skip the single-launch (lanes 1) control timing")
    ap.add_argument("--sustained-steps", type=int, default=1000,
                    help="after the K timed steps: time this many steps (SURVEY §8(d)'s 1,000) and then the same "
                         "prepared run repeated for --sustained-seconds, reported as `sustained` (0: skip)")
    ap.add_argument("--sustained-seconds", type=float, default=2.0)
    ap.add_argument("--dry-run", action="store_true", help="rank plumbing only (no GPU): every rank reports itself")
    ap.add_argument("--device-warm-ms", type=float, default=None,
                    help="ms of a VALU-bound non-step kernel (wg_launch_floor mode 2) right before the W warm-up steps "
                         "(default: WG_BENCH_WARM_MS, else 100): the GPU's clocks ramp over ~100 ms of load, and the "
                         "driver's 20-step region is shorter than that (DESIGN §6); the line reports it as "
                         "timing.device_warm_ms")
    return ap.parse_args(argv)


# ---------------------------------------------------------------- rank launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def ensure_world(args) -> None:
    """--gpus N with no torch.distributed world: start N ranks under torch.distributed.run (a child process,
    started before this process touches the GPU) and exit with its status.  A world of another size: exit 2."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
                   "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__),
                   *sys.argv[1:]]
            env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
            sys.exit(subprocess.call(cmd, env=env))
        return
    if int(world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the torch.distributed world has {world} ranks", file=sys.stderr)
        sys.exit(2)


def dry_run(args) -> None:
    """Rank plumbing without a GPU (CPU test of the launcher): gloo barrier, every rank prints itself."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    line = json.dumps({"dry_run": True, "rank": rank, "world": world, "gpus": args.gpus,
                       "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}) + "\n"
    sys.stdout.flush()
    os.write(1, line.encode())   # one write(2) per rank: ranks sharing a pipe cannot interleave inside a line
    if world > 1:
        dist.destroy_process_group()


# ---------------------------------------------------------------- workloads
def make_spec(workload: str, n: int, seed: int, chain_points: int = 100):
    from walker_gym_amd.synthetic import canonical_walkers, chain_walkers, ragged_walkers
    from walker_gym_amd.walker import balance_spec
    if workload == "canonical":
        return canonical_walkers(n, seed=seed), dict(in3d=1)
    if workload == "balance":
        return balance_spec(n), dict(in3d=0)
    if workload == "chain":      # engine.py Point.gravity (float64 anti_forced path) after the springs
        return chain_walkers(n, chain_points, seed=seed), dict(in3d=1, g=0.0, ground=-1.0e6, pair_mode=1)
    if workload == "perfdemo":   # the performance_demo loop as written: G2 Point.gravity = gravity_vec (float32)
        return chain_walkers(n, chain_points, seed=seed), dict(in3d=1, g=0.0, ground=-1.0e6, pair_mode=8)
    if workload == "lattice25":
        return canonical_walkers(n, seed=seed, M=25, K=60, A=10), dict(in3d=1)
    return ragged_walkers(n, seed=seed, mmin=4, mmax=32), dict(in3d=1)


DATA = {"canonical": "synthetic (seeded; SURVEY §8(d) canonical walker M=16, K=40, A=8; U(-1,1) actions, "
                     "distinct per step)",
        "balance": "synthetic (Balance-v0 topology, gym/optimized_walker.py:176-199; U(-1,1) actions, distinct per "
                   "step)",
        "ragged": "synthetic (seeded mixed topologies, M ~ U{4..32}, K ~ U{M..2M}, A = K // 5; U(-1,1) actions, "
                  "distinct per step)",
        "chain": "synthetic (performance_demo's chain topology: U(-100,100) positions, U(-10,10) velocities, "
                 "Skeleton(k=50) links, then gym/engine.py's Point.gravity per walker after the springs (the float64 "
                 "anti_forced path); no muscles)",
        "perfdemo": "synthetic (the performance_demo loop as written, gym/performance_demo.py:52-58, per walker: "
                    "creature.run(); Point.gravity() = optimized_engine gravity_vec (zeroes a, float32 pairs, "
                    "powf distance ** 2); Point.run1(0.01); chain topology, U(-100,100) positions, U(-10,10) "
                    "velocities)",
        "lattice25": "synthetic (seeded uniform 5x5-lattice walkers, M=25 (not a divisor of 64), K=60, A=10; U(-1,1) "
                     "actions, distinct per step)"}


def bytes_per_walker_step(host, in3d: bool) -> float:
    """SURVEY §8(d) algorithmic bytes, averaged over the batch's walkers (each walker's own M, K, A, obs row)."""
    from walker_gym_amd.layout import algorithmic_bytes_per_walker_step
    M = np.diff(host.mass_off).astype(np.int64)
    K = np.diff(host.edge_off).astype(np.int64)
    A = np.diff(host.muscle_off).astype(np.int64)
    D = 3 if in3d else 2
    obs = 3 * D * M + A
    return float(np.mean(algorithmic_bytes_per_walker_step(M, K, A, obs)))


def cpu_baseline(workload, params, chain_points, budget_s: float) -> dict:
    """The CPU side of the same workload on the box's host cores, on bounded samples:
    * reference_style: the reference's per-object numpy loop restated (oracle/refstyle.py; bit-exact with the
      goldens), single process and one spawned process per core, full env step (physics + obs/reward/done/info)
      and physics alone;
    * c_port: the C oracle (oracle/walker_oracle.c), single thread and OpenMP over walkers.
    `value` is reference_style on all cores (the reported baseline), kind "port"."""
    from oracle.oracle import Oracle
    from oracle.refstyle import host_cores, throughput
    cores = host_cores()
    pairs = workload in ("chain", "perfdemo")
    rs_n = 8 if pairs else 32
    spec = make_spec(workload, rs_n, 99, chain_points)[0]
    A = max(1, int(np.max(spec["n_muscles"])))
    acts = np.random.default_rng(123).uniform(-1, 1, (8, rs_n, A)).astype(np.float32)
    share = budget_s / 5
    rs1 = throughput(spec, params, acts, share)
    rs1p = throughput(spec, params, acts, share, observe=False)
    rsn = throughput(spec, params, acts, share, procs=cores)
    n = 512 if pairs else 4096
    spec = make_spec(workload, n, 99, chain_points)[0]
    acts = np.random.default_rng(123).uniform(-1, 1, (8, n, A)).astype(np.float32)
    res = {}
    for label, thr in (("1", 1), ("all", cores)):
        orc = Oracle(spec, params, n_threads=thr)
        t0 = time.perf_counter(); orc.step(acts[0]); probe = time.perf_counter() - t0
        steps = int(max(2, min(2000, share / max(probe, 1e-6))))
        t0 = time.perf_counter()
        for s in range(steps):
            orc.step(acts[s % 8])
        dt = time.perf_counter() - t0
        res[label] = (n * steps / dt, steps)
    return {"value": round(rsn["value"], 1), "unit": "env-steps/s", "cores": rsn["procs"], "kind": "port",
            "sample": f"{rs_n} walkers of the same workload per process, {rsn['procs']} spawned processes for "
                      f"{rsn['seconds']:.1f} s: the reference's per-object numpy loop (oracle/refstyle.py), full "
                      "env step",
            "reference_style": {"env_step_1core": round(rs1["value"], 1), "physics_only_1core": round(rs1p["value"], 1),
                                "env_step_all_cores": round(rsn["value"], 1), "procs": rsn["procs"]},
            "c_port": {"value_1core": round(res["1"][0], 1), "value_all_cores": round(res["all"][0], 1),
                       "threads": cores, "sample": f"{n} walkers x {res['all'][1]} steps, OpenMP over walkers "
                                                   "(oracle/walker_oracle.c)"}}


def load_traffic(workload: str, walkers: int):
    """HBM bytes per full-batch launch from a committed rocprofv3 PMC run (profiles/*pmc*.json), if present."""
    import glob
    best = None
    # newest round last: the round tags (r01_, r02a_, r02c_, ...) sort by name (mtimes do not survive every copy)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("workload") == workload and d.get("walkers") == walkers and "hbm_bytes_per_launch" in d:
            best = d
    return best


def clock() -> float:
    """Host CLOCK_MONOTONIC in seconds: one clock for every process of the node, so the ranks' start and end times
    compare directly (the job's span is max over ranks of t1 - min over ranks of t0)."""
    return time.clock_gettime(time.CLOCK_MONOTONIC)


class DistPlumbing:
    """The process groups of a run inside a torch.distributed world.  The default group carries the data path's
    backend: nccl (= RCCL), created with device_id so that RCCL's communicator is up before any timed region (the
    steady state of an actor that gathers every rollout), or gloo to rehearse ranks.  With nccl a second,
    gloo group carries the host-side plumbing: the barriers that open and close timed regions, the exchange of the
    ranks' clocks and identities, and the gathered-rollout checksums.  (tests/test_bench_dist.py runs it over gloo at
    world 2 and world 8.)"""

    def __init__(self, backend: str, dev):
        self.backend, self.dev, self.ctl = backend, dev, None

    def init(self) -> None:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if self.backend == "nccl":
            dist.init_process_group("nccl", device_id=self.dev)
            self.ctl = dist.new_group(backend="gloo")
        else:
            dist.init_process_group(self.backend)

    @property
    def host_group(self):
        """The gloo group for CPU tensors (None: the default group, itself gloo)."""
        return self.ctl

    def barrier(self) -> None:
        import torch.distributed as dist
        dist.barrier(group=self.ctl)

    def max_over_ranks(self, vals):
        import torch
        import torch.distributed as dist
        t = torch.tensor(vals, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ctl)
        return [float(x) for x in t.tolist()]

    def span(self, t0: float, t1: float) -> tuple:
        """(max over ranks of t1 - min over ranks of t0, max over ranks of t1 - t0): the job's time from the first rank's
        start to the last rank's end on the shared clock (start skew included), and the slowest rank's own time."""
        a, b, c = self.max_over_ranks([t1, -t0, t1 - t0])
        return a + b, c

    def comm_size(self) -> int:
        """A one-element all_reduce of ones on the default group (RCCL's communicator with nccl): the sum is the number
        of ranks the communicator actually spans."""
        import torch
        import torch.distributed as dist
        dv = self.dev if self.backend == "nccl" else torch.device("cpu")
        t = torch.ones(1, dtype=torch.float32, device=dv)
        dist.all_reduce(t)
        return int(round(float(t.item())))

    def all_objects(self, obj) -> list:
        import torch.distributed as dist
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, obj, group=self.ctl)
        return out


def comm_report(pg: "DistPlumbing", world: int, identity: dict, strict: bool) -> dict:
    """The line's `comm` block: the communicator's size (must equal the world), every rank's device
    and PCI address (the PCI addresses must be distinct when strict, i.e. RCCL; a gloo rehearsal may share one
    GPU; device indices may repeat under per-rank visibility).  A failed check ends the run with exit status 3 on every rank."""
    size = pg.comm_size()
    ids = pg.all_objects(identity)
    from walker_gym_amd.distributed import check_distinct
    distinct, why = check_distinct(ids)
    ok = size == world and (distinct or not strict)
    rep = {"backend": pg.backend, "communicator_size": size, "world": world, "ranks": ids, "distinct_devices": distinct,
           "ok": ok}
    if not ok:
        msg = f"communicator spans {size} ranks, world {world}" if size != world else why
        print(f"bench.py: comm check failed: {msg}", file=sys.stderr, flush=True)
        sys.exit(3)
    return rep


def device_warm(stream, dev, ms: float) -> float:
    """Keep the GPU busy for `ms` with a VALU-bound kernel that is not a step (wg_launch_floor mode 2, on the bench
    stream), host-synchronised every few launches; returns the time spent (s)."""
    import ctypes as C
    import torch
    from walker_gym_amd import _lib
    if ms <= 0:
        return 0.0
    L = _lib.load()
    blocks, threads = 4096, 256
    src = torch.zeros(blocks * threads, device=dev)
    dst = torch.empty_like(src)
    args = (C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()))
    sp = C.c_void_p(stream.cuda_stream)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < ms * 1e-3:
        _lib.check(L.wg_launch_floor(2, blocks, threads, *args, 4, sp), "wg_launch_floor")
        torch.cuda.synchronize()
    return time.perf_counter() - t0


def device_busy(stream, dev, launches: int) -> None:
    """Enqueue `launches` of the warm-up kernel (wg_launch_floor mode 2, ~0.1 ms each) without waiting: the GPU stays
    busy while the host waits in the barrier that opens the timed region, so the steps start at the clocks of a busy
    GPU as they do without a process group (an idle gap of a barrier's length before the clock otherwise)."""
    import ctypes as C
    import torch
    from walker_gym_amd import _lib
    blocks, threads = 4096, 256
    src = torch.zeros(blocks * threads, device=dev)
    dst = torch.empty_like(src)
    _lib.check(_lib.load().wg_launch_floor(2, blocks, threads, C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                           int(launches), C.c_void_p(stream.cuda_stream)), "wg_launch_floor")
    src.record_stream(stream)
    dst.record_stream(stream)


def host_spin(us: float) -> None:
    """Busy-wait `us` microseconds on the host: after a barrier that slept in a socket wait, the core is brought back to
    speed before the clock starts (the launch issue of the first steps runs on it)."""
    t = time.perf_counter()
    while time.perf_counter() - t < us * 1e-6:
        pass


def timed(env, acts, steps, lanes, stream):
    """Per-step kernel time with HIP events on `stream` (the calling stream waits for every walker range)."""
    import torch
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    env.run(acts, steps, lanes=lanes)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


# ---------------------------------------------------------------- main
def launch_floor(geo, stream, dev, n=2000):
    """Per-launch time (us) of an empty kernel and of a one-load-one-store kernel on the step's grid, n launches back
    to back on `stream` from one C call (wg_launch_floor, as wg_step issues a run's steps), beside a small batch's
    step: the same box's latency floor."""
    import ctypes as C
    import torch
    from walker_gym_amd import _lib
    L = _lib.load()
    blocks, threads = int(geo["blocks"]), int(geo["threads"])
    src = torch.zeros(blocks * threads, device=dev)
    dst = torch.empty_like(src)
    args = (C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()))
    sp = C.c_void_p(stream.cuda_stream)
    out = []
    for mode in (0, 1):
        _lib.check(L.wg_launch_floor(mode, blocks, threads, *args, 50, sp), "wg_launch_floor")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        _lib.check(L.wg_launch_floor(mode, blocks, threads, *args, n, sp), "wg_launch_floor")
        e1.record(stream)
        torch.cuda.synchronize()
        out.append(round(e0.elapsed_time(e1) / n * 1e3, 3))
    return out


def main():
    args = parse()
    ensure_world(args)
    if args.dry_run:
        return dry_run(args)
    import torch
    import torch.distributed as dist
    from walker_gym_amd.batched_env import BatchedPhysicsEnv
    from walker_gym_amd.distributed import gather_rollout, gather_rollout_async, rank_identity, verify_gathered
    from walker_gym_amd.layout import layout_bytes_per_walker_step

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("WG_DIST_BACKEND", "nccl")   # nccl = RCCL; gloo only to rehearse ranks on one GPU
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    # inside a torch.distributed world (WORLD_SIZE set by torch.distributed.run), world 1 included: the process group,
    # its checks and the rollout-end gather run at every N, so `torchrun --nproc-per-node 1 bench.py` executes exactly
    # the code of the 8-GPU run (RCCL init, barriers, job span over ranks, all_gather_into_tensor)
    in_world = "WORLD_SIZE" in os.environ
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    pg = DistPlumbing(backend, dev) if in_world else None
    comm = None

    def bring_up():
        # RCCL's communicator comes up here, before any timed region (the steady state of an actor that
        # gathers every rollout; the timed steps of round 5 ran before it existed), and proves its size and devices
        nonlocal comm
        pg.init()
        comm = comm_report(pg, world, dict(rank=rank, local_rank=local, **rank_identity(dev)), strict=backend == "nccl")

    # the process group comes up after the env's walker-range streams exist and have run a step: RCCL's own streams
    # then cannot take the hardware queue a side stream would otherwise get (BatchedPhysicsEnv.__init__);
    # WG_DIST_INIT_FIRST=1 (diagnostic) restores the other order
    dist_first = os.environ.get("WG_DIST_INIT_FIRST", "0") == "1"
    if in_world and dist_first:
        bring_up()

    N = args.walkers
    spec, params = make_spec(args.workload, N, seed=1000 + rank, chain_points=args.chain_points)
    env = BatchedPhysicsEnv(spec, device=dev, **params)
    A = max(1, env.batch.A)
    lanes = env._lanes(args.lanes)
    env.reserve_streams(lanes)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7 + rank)
    acts_w = (torch.rand((max(args.warmup, 1), N, A), generator=gen, device=dev) * 2 - 1).contiguous()
    acts = (torch.rand((args.steps, N, A), generator=gen, device=dev) * 2 - 1).contiguous()
    stream = torch.cuda.current_stream(dev)

    graph = env.graph(acts, args.steps, lanes=lanes) if args.graph else None
    if in_world and not dist_first:
        # one step on the walker ranges' streams binds their hardware queues before RCCL creates its own streams
        env.run(acts_w[:1], 1, lanes=lanes)
        torch.cuda.synchronize()
        bring_up()
    do_gather = in_world and not args.no_gather
    # the rollout SURVEY §8(e) gathers: every step's reward and done flags (written by the steps at per-step offsets,
    # the same bytes as overwriting one row) and the final observations
    rec = None
    dst = 0 if args.gather_to == "root" else None
    if do_gather and graph is None and args.gather != "pipelined":
        rec = {"reward": torch.empty((args.steps, N), dtype=torch.float32, device=dev),
               "done": torch.empty((args.steps, N), dtype=torch.uint8, device=dev),
               "energy": torch.empty((args.steps, N), dtype=torch.float32, device=dev),
               "centroid": torch.empty((args.steps, N, 3), dtype=torch.float32, device=dev)}

    def gather_all(obs):
        out = {"obs": gather_rollout(obs, n_total=world * N, dst=dst)}
        if rec is not None:
            out["reward"] = gather_rollout(rec["reward"], n_total=world * N, dim=1, dst=dst)
            out["done"] = gather_rollout(rec["done"], n_total=world * N, dim=1, dst=dst)
        return out

    if do_gather:
        # one untimed gather of the same tensors, so that the timed one is RCCL's steady state (its first all-gather of
        # a shape sets up buffers: 0.68 ms against 0.16-0.25 warm at world 1, profiles/r04t_nccl1)
        gather_all(env.obs)
        torch.cuda.synchronize()
    warm_ms = args.device_warm_ms if args.device_warm_ms is not None else float(os.environ.get("WG_BENCH_WARM_MS", "100"))
    warm_s = device_warm(stream, dev, warm_ms)
    if args.warmup > 0:
        env.run(acts_w, args.warmup, lanes=lanes)
    if graph is not None:
        graph.replay()                         # warm the graph path too
    # the timed call's arguments, walker ranges and C structs built here: inside the timed region the K steps are one
    # C call (run() spends ~35 us of Python before its first launch, which the GPU would idle through)
    prep = env.prepare_run(acts, args.steps, lanes=lanes, record=rec) if graph is None else None
    torch.cuda.synchronize()

    def open_region() -> float:
        # every rank: the GPU kept busy through the opening barrier (three launches of the warm-up kernel, waited for
        # below) and the host core awake after it, then synchronize; t0
        if in_world:
            if os.environ.get("WG_BENCH_BARRIER_BUSY", "1") != "0":
                device_busy(stream, dev, 3)
            pg.barrier()
            host_spin(float(os.environ.get("WG_BENCH_SPIN_US", "300")))
        torch.cuda.synchronize()
        return clock()

    def close_region(t0: float) -> tuple:
        # t1 after this rank's synchronize; the job's time = max(t1) - min(t0) over ranks on the node's shared clock,
        # then the closing barrier (its cost stays beside the figure)
        torch.cuda.synchronize()
        t1 = clock()
        if not in_world:
            return t1 - t0, t1 - t0, t1 - t0
        job, slowest = pg.span(t0, t1)
        pg.barrier()
        torch.cuda.synchronize()
        return job, slowest, pg.max_over_ranks([clock() - t0])[0]

    prev_obs = env.obs.clone() if do_gather and args.gather == "pipelined" else None
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = open_region()
    ev0.record(stream)
    pending = None
    if prev_obs is not None:
        # issued before the steps: RCCL runs it on its own stream while the walker ranges step
        pending = gather_rollout_async(prev_obs, n_total=world * N)
    if graph is not None:
        graph.replay()
    else:
        prep()
    ev1.record(stream)
    gathered = None
    if pending is not None:
        gathered = {"obs": pending.wait()}
    wall_max, slowest_rank, wall_bar_max = close_region(t0)
    step_ms = ev0.elapsed_time(ev1) / args.steps

    gather_info = None
    if do_gather:
        # the rollout-end gather (RCCL all_gather_into_tensor, shard sizes from shard_bounds) of this
        # rollout's final observations [N, D] and every step's reward and done flags [K, N], right after the barrier
        # that closes the K timed steps, timed on every rank (max): `value` is the K steps (the bench contract),
        # `value_incl_gather` the rollout with its gather.  (Pipelined, opt-in: the previous rollout's observations
        # were gathered while these K steps ran, inside the timed region; the serial gather below then adds none.)
        tg_ms = 0.0
        if pending is None:
            torch.cuda.synchronize()
            tg = clock()
            gathered = gather_all(env.obs)
            torch.cuda.synchronize()
            tg_ms = pg.max_over_ranks([clock() - tg])[0] * 1e3
            sent = {"obs": env.obs} if rec is None else {"obs": env.obs, "reward": rec["reward"], "done": rec["done"]}
        else:
            sent = {"obs": prev_obs}
        # every rank's own results must be what landed in the gathered tensors (checksums of each rank's shard)
        content = verify_gathered(sent, gathered, {"obs": 0, "reward": 1, "done": 1}, world * N, pg.host_group)
        if not content["ok"]:
            print(f"bench.py: gathered rollout does not match the ranks' own results: {content['mismatches']}",
                  file=sys.stderr, flush=True)
            sys.exit(3)
        gather_info = {"mode": args.gather, "to": ("rank 0 (dist.gather)" if dst == 0 else "every rank (all_gather)"),
                       "rows": world * N, "tensors": sorted(gathered),
                       "bytes_per_rank": int(sum(t.numel() * t.element_size() for t in sent.values())),
                       "gathered_bytes": int(world * sum(t.numel() * t.element_size() for t in sent.values())),
                       "ms": round(tg_ms, 4),
                       "value_incl_gather": round(world * N * args.steps / (wall_max + tg_ms * 1e-3), 1),
                       "content_check": content,
                       "note": "serial (default): this rollout's final observations [N, D] and its per-step reward "
                               "and done flags [K, N], gathered after the barrier closing the K timed steps, into "
                               "every rank (--gather-to root: to rank 0 only), ms = max over ranks; "
                               "value_incl_gather = the K steps and this gather; content_check: every rank's checksums "
                               "of what it sent against its shard of the gathered tensors (a mismatch exits 3); "
                               "pipelined (opt-in): the previous rollout's final observations gathered while these "
                               "steps ran (inside the timed region)"}

    # ---------------- sustained rate: the same prepared walker ranges, no extra device warm-up
    sustained = None
    B = bytes_per_walker_step(env.batch.host, bool(params.get("in3d")))
    if graph is None and args.sustained_steps > 0:
        S = args.sustained_steps
        acts_s = acts[:S] if args.steps >= S else \
            (torch.rand((S, N, A), generator=gen, device=dev) * 2 - 1).contiguous()
        prep_s = env.prepare_run(acts_s, S, lanes=lanes)
        torch.cuda.synchronize()
        runs = {}
        t0s = open_region()
        prep_s()
        j1, _, _ = close_region(t0s)
        reps = max(1, int(round(args.sustained_seconds / j1))) if args.sustained_seconds > 0 else 0
        if in_world:
            reps = int(pg.max_over_ranks([float(reps)])[0])
        runs[f"k{S}"] = (S, j1)
        if reps > 0:
            t0s = open_region()
            for _ in range(reps):
                prep_s()
            j2, _, _ = close_region(t0s)
            runs["long"] = (S * reps, j2)
        nf = None
        if os.environ.get("WG_BENCH_CHECK_FINITE", "1") != "0":
            # walkers whose state went non-finite by the end (the reference's physics diverges for some walkers under
            # random actions; their waves then run the exact IEEE cold paths): counted, so the figure says what it timed
            bad = ~(torch.isfinite(env.batch.pos).all(1) & torch.isfinite(env.batch.vel).all(1))
            wid = torch.from_numpy(np.repeat(np.arange(env.N), np.diff(env.batch.host.mass_off))).to(dev)
            nf = int(torch.zeros(env.N, dtype=torch.int32, device=dev).index_put_((wid,), bad.int(), accumulate=True)
                     .gt(0).sum().item())
        head_v = world * N * args.steps / wall_max
        sustained = {}
        for key, (steps_, sec) in runs.items():
            ms = sec * 1e3 / steps_
            ach = B * N / (ms * 1e-3) / 1e9
            sustained[key] = {"steps": steps_, "seconds": round(sec, 4), "ms_per_step": round(ms, 5),
                              "value": round(world * N * steps_ / sec, 1), "achieved": round(ach, 1),
                              "frac": round(ach / HBM_PEAK_GBS, 4)}
        last = sustained["long" if "long" in sustained else f"k{S}"]
        sustained["burst_over_sustained"] = round(head_v / last["value"], 4)
        sustained["nonfinite_walkers_at_end"] = nf
        sustained["note"] = (f"after the K timed steps, in the same process: {S} steps (SURVEY §8(d)'s region) and then "
                             f"the same {S}-step prepared run repeated back to back for ~{args.sustained_seconds:g} s "
                             "('long'), with the headline's walker ranges and no extra device warm-up; job time as the "
                             "headline (max over ranks of t1 - min of t0).  achieved / frac: N * B / ms_per_step (the "
                             "two-range step) against 8 TB/s.  burst_over_sustained = value / long.value: the driver's "
                             "K = 20 region runs at the GPU's burst clock, a long run at its sustained clock (DESIGN §6)."
                             + (" Outputs overwritten each step (no per-step records)." if rec is not None else ""))

    if rank == 0:
        # single-launch control: one full-batch launch per step, HIP events on its stream — the per-dispatch
        # duration a rocprofv3 kernel trace of `bench.py --lanes 1` reports (profiles/*_kernel_groups.json)
        # (200 launches with their own distinct actions whatever K is: at a short K the first launches of a process
        # still see the clocks ramp, and the per-launch figure is the kernel's, not the bench's K)
        n1 = 200
        single_ms = step_ms if (lanes == 1 and graph is None and args.steps >= n1) else None
        acts_c = acts[:n1] if args.steps >= n1 else \
            (torch.rand((n1, N, A), generator=gen, device=dev) * 2 - 1).contiguous()
        if single_ms is None and not args.no_control:
            env.run(acts_c, n1, lanes=1)
            single_ms = timed(env, acts_c, n1, 1, stream)
        # the kernel's own duration: the same 200 launches, each one's start and end stamped on HIP events of its own by
        # the dispatch (wg_time_step: hipExtLaunchKernel, the timestamps a rocprofv3 kernel trace reports), so the gaps
        # between back-to-back dependent launches are not counted (single_ms above counts them)
        kern_ms, kern_err = None, None
        if not args.no_control:
            try:   # (a measurement aid: the line still prints, with the back-to-back figure, if it is unavailable)
                kern_ms = env.time_launches(acts_c, n1)
            except Exception as e:  # noqa: BLE001
                kern_err = f"{type(e).__name__}: {e}"
        direct_ms = timed(env, acts, args.steps, lanes, stream) if graph is not None else None
        # closed loop: one BatchedPhysicsEnv.step per env step, as a policy loop calls it (the walker ranges join
        # at the end of every step, and every step returns obs/reward/done/info); the headline `value` instead
        # issues the K steps back to back (open loop: actions known up front, ranges drift out of phase)
        closed_ms = None
        open_ms = None
        if not args.no_control:
            n_cl = n1
            for s_ in range(5):
                env.step(acts_c[s_])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for s_ in range(n_cl):
                env.step(acts_c[s_])
            e1.record(stream)
            torch.cuda.synchronize()
            closed_ms = e0.elapsed_time(e1) / n_cl
            # the open loop over the same 200-step region the closed loops below are timed on (VERDICT r5 item 1:
            # like with like), the headline's walker ranges and prepared call
            prep_c = env.prepare_run(acts_c, n1, lanes=lanes)
            prep_c()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            prep_c()
            e1.record(stream)
            torch.cuda.synchronize()
            open_ms = e0.elapsed_time(e1) / n1
        # closed loop with a policy (every action a function of the current observation): a row-wise policy, tanh of
        # each walker's observed muscle lengths, driven (a) by step() in a loop — one barrier per step — and (b) by
        # policy_loop, the walker ranges pipelined (each range acts on its own rows and steps on its own stream);
        # (a) and (b) give bit-identical trajectories
        policy_cl = None
        if not args.no_control and args.workload not in PAIR_FLOP:
            Acols = env.batch.A
            if env.batch.ragged:   # (a ragged row is zero padded past its own muscles: its first A columns instead)
                pol = lambda rows, t: torch.tanh(rows[:, :Acols])
            else:
                pol = lambda rows, t: torch.tanh(rows[:, rows.shape[1] - Acols:])
            for _ in range(3):
                env.step(pol(env.obs, 0))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for s_ in range(n1):
                env.step(pol(env.obs, s_))
            e1.record(stream)
            torch.cuda.synchronize()
            step_pol_ms = e0.elapsed_time(e1) / n1
            env.policy_loop(pol, 5, lanes=lanes)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            env.policy_loop(pol, n1, lanes=lanes)
            e1.record(stream)
            torch.cuda.synchronize()
            ranges_ms = e0.elapsed_time(e1) / n1
            # the loop's own cost: the same policy_loop with a policy that launches nothing (preallocated actions of
            # each range's row count), so the difference to the open loop is the loop's host issue and per-range checks
            null_acts = {}

            def pol_null(rows, t):
                a = null_acts.get(rows.shape[0])
                if a is None:
                    a = null_acts[rows.shape[0]] = torch.zeros((rows.shape[0], Acols), device=dev)
                return a
            env.policy_loop(pol_null, 5, lanes=lanes)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            env.policy_loop(pol_null, n1, lanes=lanes)
            e1.record(stream)
            torch.cuda.synchronize()
            null_ms = e0.elapsed_time(e1) / n1
            env.policy_loop(pol, 5, lanes=lanes, graph=True)    # warm the capture path
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            env.policy_loop(pol, n1, lanes=lanes, graph=True)   # (capture on the host, then one replay)
            torch.cuda.synchronize()
            g = env._policy_graph
            e0.record(stream)
            g.replay()
            e1.record(stream)
            torch.cuda.synchronize()
            ranges_graph_ms = e0.elapsed_time(e1) / n1
            policy_cl = {"policy": ("action = tanh(the walker's own observed muscle lengths), one elementwise kernel "
                                    "per call (row-wise)") if not env.batch.ragged else
                                   ("action = tanh(the first A columns of the walker's own observation row), row-wise; "
                                    "policy_loop splits the ranges where their walkers are caller-contiguous (a range "
                                    "elsewhere gathers its rows and scatters its actions)"),
                         "steps": n1,
                         "open_loop_ms_per_step": round(open_ms, 5),
                         "step_loop_ms_per_step": round(step_pol_ms, 5),
                         "policy_loop_ms_per_step": round(ranges_ms, 5),
                         "policy_loop_graph_ms_per_step": round(ranges_graph_ms, 5),
                         "policy_loop_null_policy_ms_per_step": round(null_ms, 5),
                         "policy_loop_over_open_loop": round(ranges_ms / open_ms, 4),
                         "lanes": lanes,
                         "note": "every figure over the same 200-step region (HIP events): open_loop: the prepared run "
                                 "of the headline's walker ranges with the actions known up front; step_loop: "
                                 "BatchedPhysicsEnv.step(policy(obs)) per env step (a full barrier per step: each "
                                 "launch drains alone); policy_loop: the walker ranges pipelined, each range's policy "
                                 "and step on its own stream (bit-identical trajectories, tests/test_gpu_policy_loop.py); "
                                 "graph: the same loop captured as one HIP graph per walker range, each replayed on its "
                                 "own stream; null_policy: policy_loop with a policy that launches nothing (the loop's "
                                 "own cost against the open loop)"}
        resident_ms = None
        if args.resident:
            env.run(acts_c, n1, lanes=1, resident=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            env.run(acts, args.steps, lanes=1, resident=True)
            e1.record(stream)
            torch.cuda.synchronize()
            resident_ms = e0.elapsed_time(e1) / args.steps
        D = env.obs_dim
        M, K = env.batch.M, env.batch.K
        uniform = not env.batch.ragged
        if uniform:
            B_layout = layout_bytes_per_walker_step(M, K, env.batch.A, D)
        else:   # per walker (its own M, K, A and obs row), averaged; the buffer-by-buffer account is DESIGN §4
            hm = env.batch.host
            Mw, Kw, Aw = np.diff(hm.mass_off), np.diff(hm.edge_off), np.diff(hm.muscle_off)
            B_layout = round(float(np.mean(layout_bytes_per_walker_step(
                Mw, Kw, Aw, (9 if params.get("in3d") else 6) * Mw + Aw, ragged=True))), 1)
        tr = load_traffic(args.workload, N)
        geo = env.launch_geometry()
        bb_ms = single_ms if single_ms is not None else step_ms
        head_ms = kern_ms if kern_ms is not None else bb_ms
        achieved = B * N / (head_ms * 1e-3) / 1e9
        line = {
            "metric": METRIC,
            "value": round(world * N * args.steps / wall_max, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max * 1e3 / args.steps, 5),
            "timing": {"clock": ("host CLOCK_MONOTONIC, one clock for the node's ranks: t0 after the opening barrier + "
                                 "synchronize, t1 after each rank's synchronize; job time = max(t1) - min(t0) over "
                                 "ranks (start skew included)" if in_world else
                                 "host CLOCK_MONOTONIC: t0 after synchronize, t1 after synchronize"),
                       "ms_per_step_slowest_rank": round(slowest_rank * 1e3 / args.steps, 5),
                       "ms_per_step_incl_closing_barrier": round(wall_bar_max * 1e3 / args.steps, 5),
                       "device_warm_ms": round(warm_s * 1e3, 2),
                       "kernel_ms_per_step_events": round(step_ms, 5),
                       "region": "burst: a K-step region after a 100 ms device warm-up runs at the GPU's burst clock; "
                                 "`sustained` times 1,000 steps and a ~2 s run of the same walker ranges beside it",
                       **({"comm": "RCCL's communicator up before the timed steps (created and checked by a one-element "
                                   "all_reduce, then one untimed gather of the rollout's tensors); barriers and the "
                                   "clock exchange on a gloo group"} if in_world and backend == "nccl" else
                          {"comm": f"{backend} process group (rehearsal, no RCCL)"} if in_world else {})},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": DATA[args.workload],
            "config": {"workload": f"{args.workload} walkers, {N} per GPU (M={M}{'' if uniform else ' max'}, "
                                   f"K={K}{'' if uniform else ' max'}, A={env.batch.A}, obs D={D}), one fused "
                                   "act+physics+observe launch per env step per walker range "
                                   f"({lanes} range{'s' if lanes > 1 else ''} on {lanes} stream{'s' if lanes > 1 else ''})"
                                   + (", replayed as one HIP graph" if graph is not None else ""),
                       "walkers_per_gpu": N, "total_walkers": world * N, "M": M, "K": K, "A": env.batch.A,
                       "obs_dim": D, "parallelism": f"dp{world}",
                       "rollout_gather": (args.gather if gathered is not None else False),
                       "dist_backend": (dist.get_backend() if in_world else None),
                       **({"dist_init": "before the env" if dist_first else "after the env's streams and first step"}
                          if in_world else {}),
                       "lanes": lanes, "launch": geo, "ragged_kind": env.batch.ragged_kind,
                       **({"chain_points": args.chain_points, "pair_mode": params["pair_mode"]}
                          if args.workload in PAIR_FLOP else {})},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": (tr["hbm_bytes_per_launch"] if tr else None),
                         "bytes_per_walker_step": round(B, 1), "layout_bytes_per_walker_step": B_layout,
                         "kernel_ms_per_launch": round(head_ms, 5),
                         **({"ms_per_launch_back_to_back": round(bb_ms, 5)} if kern_ms is not None else {}),
                         **({"wg_time_step_error": kern_err} if kern_err else {}),
                         "note": ("achieved = N * B / the mean duration of ONE full-batch launch (200 launches, one "
                                  "per step, each launch's own start and end stamped on HIP events by the dispatch: "
                                  "wg_time_step / hipExtLaunchKernel, the timestamps a rocprofv3 --kernel-trace of this "
                                  "command reports for the full-grid launches, scripts/trace_kernels.py); "
                                  "ms_per_launch_back_to_back: the same launches timed by two events around all 200 "
                                  "(the gaps between dependent launches included); B = SURVEY §8(d) algorithmic bytes "
                                  "averaged over the walkers") if kern_ms is not None else
                                 ("achieved = N * B / the per-launch time of ONE full-batch launch per step (HIP "
                                  "events around back-to-back launches on the launching stream); B = SURVEY §8(d) "
                                  "algorithmic bytes averaged over the walkers") if single_ms is not None else
                                 (f"achieved = N * B / the time per step of the {lanes} walker ranges (--no-control: "
                                  "no single-launch timing); B = SURVEY §8(d) algorithmic bytes averaged over the "
                                  "walkers")},
        }
        if comm is not None:
            line["comm"] = comm
        if sustained is not None:
            line["sustained"] = sustained
        if lanes > 1 or graph is not None:
            a2 = B * N / (step_ms * 1e-3) / 1e9
            line["roofline"]["concurrent"] = {
                "lanes": lanes, "kernel_ms_per_step_events": round(step_ms, 5), "achieved": round(a2, 1),
                "frac": round(a2 / HBM_PEAK_GBS, 4),
                "note": f"{lanes} walker ranges on {lanes} streams overlap one range's launch tail with the other's "
                        "next step: HIP events around the K timed steps (burst region; `sustained` has the long-run "
                        "fraction)"}
        if graph is not None:
            line["graph"] = {"replay_ms_per_step": round(step_ms, 5), "direct_ms_per_step": round(direct_ms, 5),
                             "launch_overhead_share": round(max(0.0, 1 - step_ms / direct_ms), 4)}
        if closed_ms is not None:
            line["closed_loop"] = {
                "ms_per_step": round(closed_ms, 5), "env_steps_per_s": round(N * 1e3 / closed_ms, 1),
                "open_loop_ms_per_step": round(open_ms, 5),
                "lanes": env._step_lanes(),
                "note": "BatchedPhysicsEnv.step() once per env step (HIP events on the calling stream over 200 "
                        "steps; one walker range, step()'s default): each step returns obs / reward / done / info "
                        "— what a PhysicsEnv.step caller gets; open_loop: the headline's prepared walker ranges over "
                        "the same 200 steps"}
        if policy_cl is not None:
            line["closed_loop_policy"] = policy_cl
        if resident_ms is not None:
            line["resident_rollout"] = {
                "ms_per_step": round(resident_ms, 5), "env_steps_per_s": round(N * 1e3 / resident_ms, 1),
                "lanes": 1,
                "note": "the same K steps as ONE wg_rollout launch: each wave's walker state in registers across steps, "
                        "per-step obs/reward/done/info written every step (open-loop actions known up front); not the "
                        "headline, which is one launch per env step (SURVEY 8(d))"}
        if tr:
            line["roofline"]["traffic_source"] = tr.get("source")
        if args.workload in PAIR_FLOP:
            # O(M^2) per walker: the partner loops, not HBM, bound these launches; the roofline is the VALU's
            flop_pair, bound, peak = PAIR_FLOP[args.workload]
            pairs = N * args.chain_points * (args.chain_points - 1) / 2
            tfs = pairs * flop_pair / (head_ms * 1e-3) / 1e12
            hbm = dict(line["roofline"])
            line["roofline"] = {"bound": bound, "achieved": round(tfs, 3), "peak": peak, "unit": "TFLOP/s",
                                "frac": round(tfs / peak, 4), "traffic": hbm.get("traffic"),
                                "flop_per_pair": flop_pair, "pairs_per_launch": int(pairs),
                                "flop_per_launch": int(pairs * flop_pair), "kernel_ms_per_launch": round(head_ms, 5),
                                "note": ("achieved = the reference pair loop's algorithmic FLOP per unordered pair x "
                                         "the pairs of one launch (N * M(M-1)/2) / the mean duration of ONE "
                                         "full-batch launch (HIP events stamped by the dispatch, wg_time_step); peak = "
                                         "the vector "
                                         + ("FP64" if bound == "fp64-valu" else "FP32") + " rate (bench.py "
                                         "FP64_PEAK_TFS / FP32_PEAK_TFS, measured by scripts/valu_peak.hip)"),
                                "hbm": {k: hbm[k] for k in ("achieved", "peak", "unit", "frac", "bytes_per_walker_step")}}
            line["pairs_per_s"] = round(pairs / (head_ms * 1e-3), 1)
        if N <= 16384:
            # a small batch is one wave's latency chain per launch: state the launch floor it is bounded by, timed
            # here, on this box and stream, for the step's own grid (wg_launch_floor: back-to-back launches of an
            # empty kernel and of one coalesced load + store per thread, HIP events)
            fl = launch_floor(geo, stream, dev)
            line["floor"] = {"empty_launch_us": fl[0], "load_store_launch_us": fl[1],
                             "step_over_load_store": round(step_ms * 1e3 / fl[1], 3),
                             "kernel_over_load_store": round(bb_ms * 1e3 / fl[1], 3),   # (both back to back)
                             # --resident: the same steps as one wg_rollout launch (no launch per step)
                             **({"resident_step_over_load_store": round(resident_ms * 1e3 / fl[1], 3)}
                                if resident_ms is not None else {}),
                             "grid": [geo["blocks"], geo["threads"]],
                             "source": "wg_launch_floor on this box (the step's grid, 2,000 back-to-back launches "
                                       "each, HIP events on the bench stream); scripts/launch_floor.hip is the "
                                       "standalone form (profiles/r03_launch_floor.json)"}
        if gather_info is not None:
            line["gather"] = gather_info
            # BASELINE config 4 includes the rollout-end gather: its figure, beside the steps-only `value`
            line["value_incl_gather"] = gather_info["value_incl_gather"]
            line["value_definition"] = ("value: the K timed steps alone (the bench contract times exactly K steps between "
                                        "two barriers); value_incl_gather: BASELINE config 4 as defined — the K steps "
                                        "and the rollout-end RCCL gather of the final observations and every step's "
                                        "reward and done flags (gather.ms, max over ranks)")
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.workload, params, args.chain_points, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if in_world:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
