"""libwalker_hip's host code under AddressSanitizer: the library rebuilt with -Xarch_host -fsanitize=address (device
code unoptimised, it is never launched here) and scripts/host_asan_check.c driving the planners, their error paths,
launch geometry and argument validation on seeded ragged batches in exactly-sized buffers."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
CLANG = "/opt/rocm/lib/llvm/bin/clang"


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(CLANG)), reason="no ROCm toolchain")
def test_library_host_code_under_asan(tmp_path):
    lib = tmp_path / "libwalker_hip_asan.so"
    inc = os.path.join(ROOT, "include")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-Xarch_host",
                    "-fsanitize=address", "-Xarch_device", "-O0", "-Wno-pass-failed", "-I", inc, "-o", str(lib),
                    os.path.join(ROOT, "walker_gym_amd", "csrc", "walker_hip.hip")], check=True, capture_output=True,
                   timeout=600)
    drv = tmp_path / "host_asan_check"
    subprocess.run([CLANG, "-fsanitize=address", "-g", "-I", inc, "-o", str(drv),
                    os.path.join(ROOT, "scripts", "host_asan_check.c"), f"-L{tmp_path}", "-lwalker_hip_asan",
                    f"-Wl,-rpath,{tmp_path}"], check=True, capture_output=True, timeout=120)
    r = subprocess.run([str(drv)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))   # the HIP runtime's own allocations
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "host asan ok" in r.stdout
