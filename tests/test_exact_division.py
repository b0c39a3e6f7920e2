"""The kernel's exact-quotient identities (walker_hip.hip fdiv_exact / ddiv_exact), checked on the host
with the same IEEE arithmetic: 0 mismatches over random and adversarial operands."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exact_division_identities(tmp_path):
    exe = tmp_path / "check_division"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(ROOT, "scripts", "check_division.c"),
                    "-lm"], check=True)
    r = subprocess.run([str(exe), "4000000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "bad f32-via-f64=0 markstein(t/m)=0 markstein(fv/c)=0" in r.stdout
    assert "adversarial bad=0" in r.stdout
    assert "count-divisor" in r.stdout and "count-divisor n=" in r.stdout
    lines = {l.split()[0]: l for l in r.stdout.splitlines()}
    assert lines["count-divisor"].endswith("bad=0") and lines["exact-range"].endswith("bad=0")
