#!/usr/bin/env python3
"""Resource usage (VGPRs, scratch, occupancy) of every kernel in walker_hip.hip:
    python scripts/kres.py [extra hipcc flags, e.g. -DWG_LEAN_SOA=0]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero", "-mllvm",
       "-amdgpu-kernarg-preload-count=10", "--cuda-device-only", "-c",
       "-Rpass-analysis=kernel-resource-usage", "-I", os.path.join(ROOT, "include"), "-o", "/dev/null", *sys.argv[1:],
       os.path.join(ROOT, "walker_gym_amd", "csrc", "walker_hip.hip")]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = {}, None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = re.sub(r"\(anonymous namespace\)::", "", cur).split("(")[0]
        rows[cur] = {}
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur:
            rows[cur][key] = int(m.group(1))
for k, v in rows.items():
    print(f"{k:60s} vgpr {v.get('vgpr'):4} scratch {v.get('scratch'):4} occ {v.get('occ')}")
