#!/usr/bin/env python3
"""Time several builds of libwalker_hip.so on the canonical 65,536-walker step, alternating processes
over rounds (experiment aid).  usage: python scripts/rev_ab.py ROUNDS LIB..."""
import subprocess
import sys

rounds, libs = int(sys.argv[1]), sys.argv[2:]
res = {l: [] for l in libs}
for r in range(rounds):
    for l in libs:
        out = subprocess.run([sys.executable, "scripts/ablate.py", "one", l], capture_output=True, text=True, timeout=300)
        res[l].append(out.stdout.strip() or out.stderr.strip()[-200:])
        print(r, l, res[l][-1], flush=True)
