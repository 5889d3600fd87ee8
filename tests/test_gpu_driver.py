"""The C++ drivers over the C ABI on the GPU (SURVEY 8b caller contracts, 8f).

./multigrid (driver/multigrid.cpp) with the reference's defaults at N=32 must
write uT.txt and uTomp.txt byte-identical to the reference's own result in
the reference's format (tests/golden/uT_N32.txt), print the reference's
lines, and report zero difference between its op-level control flow and the
library's fast path.  ./mg_sweep writes cudatime.txt / gpups.txt in the
"N<TAB>value" format speedupplot.py reads.
"""
import os
import re
import subprocess

import pytest
from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu


def _built(name):
    exe = os.path.join(ROOT, name)
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "driver")], check=True)
    return exe


def test_multigrid_driver_writes_reference_uT(tmp_path):
    exe = _built("multigrid")
    out = subprocess.run([exe, "-N", "32", "-out", str(tmp_path) + "/"], capture_output=True,
                         text=True, timeout=300, check=True).stdout
    with open(os.path.join(GOLDEN, "uT_N32.txt")) as f:
        want = f.read()
    for name in ("uT.txt", "uTomp.txt"):
        with open(tmp_path / name) as f:
            assert f.read() == want, name
    # the reference's line shapes (multigrid.cpp:246, :259, :266), labelled
    # with what ran (both legs on the GPU), then the %10e error line
    lines = out.split("\n")
    timed = [l for l in lines if re.fullmatch(r".+ time, N = 32: \d+\.\d{6} s", l)]
    assert len(timed) == 2, out
    assert re.fullmatch(r"GPU \(reference op sequence, 1 MI355X\) time, N = 32: \d+\.\d{6} s",
                        timed[0])
    assert re.fullmatch(r"GPU \(mgx_timestepper fused passes, 1 MI355X\) time, N = 32: "
                        r"\d+\.\d{6} s", timed[1])
    assert lines[lines.index(timed[0]) - 1] == "" and lines[lines.index(timed[1]) - 1] == ""
    assert "Error (compared to the referenced solution) = 0.000000e+00" in lines


def test_multigrid_driver_fma_mode(tmp_path):
    """./multigrid -fp fma: run 2 (the library's time stepper) contracted; its
    L1 distance from run 1 (the bitwise op-level sequence) over the N=128
    grid stays within (N+1)^2 x 1e-12 and is not zero."""
    exe = _built("multigrid")
    out = subprocess.run([exe, "-N", "128", "-fp", "fma", "-out", str(tmp_path) + "/"],
                         capture_output=True, text=True, timeout=300, check=True).stdout
    m = re.search(r"Error \(compared to the referenced solution\) = (\S+)", out)
    err = float(m.group(1))
    assert 0.0 < err <= 129 * 129 * 1e-12, out


def test_mg_sweep_formats(tmp_path):
    exe = _built("mg_sweep")
    out = subprocess.run([exe, "-Nmin", "32", "-Nmax", "256", "-cycles", "2", "-steps", "5",
                          "-out", str(tmp_path) + "/"], capture_output=True, text=True,
                         timeout=300, check=True).stdout
    assert out.count("Time elapsed for grid size") == 4
    for name, conv in (("cudatime.txt", float), ("gpups.txt", float)):
        rows = [l.split("\t") for l in open(tmp_path / name).read().splitlines()]
        assert [int(r[0]) for r in rows] == [32, 64, 128, 256]
        assert all(conv(r[1]) > 0 for r in rows)


def test_bench_sweep_writes_speedupplot_inputs(tmp_path):
    """bench.py --sweep: cudatime.txt / serialtime.txt / omptime.txt in the
    'N<TAB>seconds' format speedupplot.py reads (/root/reference/speedupplot.py
    :10,25,40); the GPU and the reference's serial and OpenMP runs agree bitwise."""
    import json
    import sys
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--sweep", "32", "64",
                          "--sweep-out", str(tmp_path) + "/"], capture_output=True, text=True,
                         timeout=300, check=True).stdout
    rec = json.loads(out.strip().splitlines()[-1])
    assert [r["N"] for r in rec["sweep"]] == [32, 64]
    assert all(r["serial_bitwise"] and r["omp_bitwise"] for r in rec["sweep"])
    for name in ("cudatime.txt", "serialtime.txt", "omptime.txt"):
        rows = [l.split("\t") for l in open(tmp_path / name).read().splitlines()]
        assert [int(r[0]) for r in rows] == [32, 64]
        assert all(float(r[1]) > 0 for r in rows)
