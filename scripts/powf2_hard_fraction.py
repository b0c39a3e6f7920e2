#!/usr/bin/env python3
"""How often numpy's x ** 2 needs the restated powf (profiling aid, not product): the fraction of the performance_demo
chains' partner distances whose square lies inside pw_pow2_fast's band (powf2.h), new and old, and the chance that a
64-lane wave's partner iteration holds at least one such lane.  Run from the repo root: python scripts/powf2_hard_fraction.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from walker_gym_amd.synthetic import chain_walkers
s = chain_walkers(64, 100, seed=1)
P = s['pos'].reshape(64, 100, 3).astype(np.float32)
d = P[:, :, None, :] - P[:, None, :, :]
sq = (d.astype(np.float64) ** 2).sum(-1).astype(np.float32)
dist = np.sqrt(sq).astype(np.float32)          # ~ sqrt_mid (correctly rounded)
x = dist[dist > 0].astype(np.float64)
e = x * x
E = np.frexp(e)[1]
dband = np.ldexp(1.75e-3, E - 24)
lo = (e - dband).astype(np.float32); hi = (e + dband).astype(np.float32)
hard = lo != hi
print('fraction hard (new band):', hard.mean())
dold = e * 2.0**-32
hard_old = (e - dold).astype(np.float32) != (e + dold).astype(np.float32)
print('fraction hard (old band):', hard_old.mean())
p = hard.mean(); print('P(wave iteration has a cold lane) ~', 1 - (1 - p) ** 64)
