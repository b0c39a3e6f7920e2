"""Build libwalker_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m walker_gym_amd.build [--force] [--verbose]

Numerics-relevant flags (the kernel restates numpy's float semantics op by op):
  -ffp-contract=off                        no a*b+c -> fma fusion (numpy rounds every op)
  -fhip-fp32-correctly-rounded-divide-sqrt IEEE float32 '/' and sqrtf
  -fno-gpu-flush-denormals-to-zero         keep float32 denormals, as x86 SSE does
and one performance flag: -mllvm -amdgpu-kernarg-preload-count=10 (walker_step_lean1's leading arguments in SGPRs).
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "walker_hip.hip")
HDR = os.path.join(ROOT, "include", "walker_hip.h")
POWF2 = os.path.join(HERE, "csrc", "powf2.h")
OUT = os.path.join(HERE, "libwalker_hip.so")
ARCH = os.environ.get("WALKER_HIP_ARCH", "gfx950")

FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
         # the NE = 1 step kernel's ten leading arguments preloaded into SGPRs by the dispatch (walker_step_lean1;
         # kernels whose first argument is a struct get none)
         "-mllvm", "-amdgpu-kernarg-preload-count=10",
         "-Wall", "-Wno-unused-function"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm 7.x expected at /opt/rocm)")


def command(out: str = OUT) -> list:
    return [hipcc(), f"--offload-arch={ARCH}", *FLAGS, "-I", os.path.join(ROOT, "include"), "-o", out, SRC]


def needs_build(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in (SRC, HDR, POWF2, __file__))


def build(force: bool = False, verbose: bool = False) -> str:
    if force or needs_build():
        cmd = command()
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build(a.force, a.verbose))


if __name__ == "__main__":
    sys.exit(main())
