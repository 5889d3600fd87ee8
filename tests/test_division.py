"""The smoother divides by the diagonal with a reciprocal + one Markstein
correction (kernels.hip div_diag).  This checks on the host, with the same
instruction sequence (fma from libm), that it is bitwise IEEE division for
every diagonal the solver uses and for random divisors."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_markstein_division_is_correctly_rounded(tmp_path):
    exe = tmp_path / "check_division"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tools", "check_division.c"), "-lm"], check=True)
    out = subprocess.run([str(exe), "300000", "20000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "mismatches 0" in out.stdout
