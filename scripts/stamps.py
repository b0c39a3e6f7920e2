#!/usr/bin/env python3
"""Phase timeline of the lean kernel (or, WG_WORKLOAD=ragged, the ragged wave kernel) from a -DWG_STAMPS build
(profiling aid, not product).

    python scripts/variant_ab.py build stamps=-DWG_STAMPS     # here
    python scripts/stamps.py [ab_session/lib_stamps.so]         # GPU box: one full-batch canonical launch

Stamps (s_memtime, shader clock) per wave: 0 entry, 1 loads issued, 2 loads landed + act done, 3 springs done,
4 masses + integrator done, 5 reductions + state stores issued, 6 obs streamed.  Prints the mean phase durations,
the wave start / end spread and the live-wave count over the launch; writes gpurun_out/stamps.json."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["WALKER_HIP_LIB"] = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "ab_session", "lib_stamps.so")
import torch  # noqa: E402

from bench import make_spec  # noqa: E402
from walker_gym_amd import _lib  # noqa: E402
from walker_gym_amd.batched_env import BatchedPhysicsEnv  # noqa: E402

N = int(os.environ.get("WG_N", "65536"))
WORKLOAD = os.environ.get("WG_WORKLOAD", "canonical")     # canonical (lean kernel) or ragged (wave kernel)
spec, params = make_spec(WORKLOAD, N, seed=1000)
env = BatchedPhysicsEnv(spec, device="cuda:0", **params)
acts = (torch.rand((60, N, max(1, env.batch.A)), device="cuda:0") * 2 - 1).contiguous()
env.run(acts[:50].contiguous(), 50, lanes=1)          # past the free fall, as in the bench's timed region
env.run(acts[50:51].contiguous(), 1, lanes=1)
torch.cuda.synchronize()
geo = env.batch.launch_geometry()
wpw = geo["walkers_per_block"] // max(1, geo["threads"] // 64)   # walkers per wave tile (lean kernel)
W = env.batch.plan_blocks if env.batch.ragged else -(-N // wpw)     # waves (one tile each)
st = np.zeros((W, 8), np.uint64)
print("WG_LEAN_WAVES", os.environ.get("WG_LEAN_WAVES", "auto"))
L = _lib.load()
L.wg_debug_stamps.argtypes = [C.c_void_p, C.c_int]
assert L.wg_debug_stamps(st.ctypes.data_as(C.c_void_p), W) == 0
t = st[:, :7].astype(np.int64)
hw = st[:, 7].astype(np.int64)
xcc = (hw >> 32) & 0xF
se = (hw >> 13) & 0x7
sh = (hw >> 12) & 0x1
cu = (hw >> 8) & 0xF
cukey = ((xcc * 8 + se) * 2 + sh) * 16 + cu
# s_memtime is not one clock across the chip: align each CU (its own counter) to its first wave start
for x in np.unique(cukey):
    sel = cukey == x
    t[sel] -= t[sel, 0].min()
ph = np.diff(t, axis=1)
names = ["issue loads", "load wait + act", "springs", "masses + tail", "reduce + store", "obs"]
out = {"waves": W, "clock": "s_memtime cycles"}
for i, nme in enumerate(names):
    out[nme] = {"mean": float(ph[:, i].mean()), "p50": float(np.median(ph[:, i])), "p90": float(np.percentile(ph[:, i], 90)),
                "p99": float(np.percentile(ph[:, i], 99)), "max": float(ph[:, i].max())}
simd = (hw >> 4) & 0x3
out["waves_per_simd"] = [int((simd == k).sum()) for k in range(4)]
first = t[:, 0] < 2000                       # the CU's first round (it starts idle)
out["first_round"] = {nme: float(ph[first, i].mean()) for i, nme in enumerate(names)}
out["later_rounds"] = {nme: float(ph[~first, i].mean()) for i, nme in enumerate(names)}
life = t[:, 6] - t[:, 0]
# the compute phases only (springs .. obs: stamps 2 -> 6), free of the load latency and of clock alignment
comp = t[:, 6] - t[:, 2]
out["compute_lifetime"] = {"p50": float(np.median(comp)), "p90": float(np.percentile(comp, 90)),
                           "p99": float(np.percentile(comp, 99)), "max": float(comp.max())}
out["lifetime"] = {"mean": float(life.mean()), "p50": float(np.median(life)), "p90": float(np.percentile(life, 90))}
out["span"] = int(t[:, 6].max())
out["start_p"] = [int(np.percentile(t[:, 0], q)) for q in (0, 10, 50, 90, 100)]
out["end_p"] = [int(np.percentile(t[:, 6], q)) for q in (0, 10, 50, 90, 100)]
edges = np.linspace(0, out["span"], 41)
live = [int(((t[:, 0] <= x) & (t[:, 6] > x)).sum()) for x in edges[:-1]]
out["live_waves"] = live
out["xcds"] = int(len(np.unique(xcc)))
out["cus"] = int(len(np.unique(cukey)))
spans = np.array([t[cukey == x, 6].max() for x in np.unique(cukey)])
out["cu_span_p"] = [int(np.percentile(spans, q)) for q in (0, 10, 50, 90, 100)]
waves_cu = np.array([(cukey == x).sum() for x in np.unique(cukey)])
out["waves_per_cu_p"] = [int(np.percentile(waves_cu, q)) for q in (0, 50, 100)]
per = {}
for x in np.unique(cukey)[:6]:
    sel = cukey == x
    tt = t[sel]
    per[int(x)] = {"waves": int(sel.sum()), "span": int(tt[:, 6].max()),
                   "start_p": [int(np.percentile(tt[:, 0], q)) for q in (0, 10, 50, 90, 100)],
                   "end_p": [int(np.percentile(tt[:, 6], q)) for q in (0, 10, 50, 90, 100)],
                   "live": [int(((tt[:, 0] <= y) & (tt[:, 6] > y)).sum())
                            for y in np.linspace(0, tt[:, 6].max(), 33)[:-1]]}
out["per_xcd"] = per
print(json.dumps(out, indent=1))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", os.environ.get("WG_STAMPS_OUT", "stamps.json")), "w"), indent=1)
