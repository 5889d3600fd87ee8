"""Output formats the reference's scripts read (SURVEY 8b caller contracts).

uT.txt / uTomp.txt / uTcuda.txt: "%d\t%d\t%f\n", i outer, j inner, (N+1)^2
lines (multigrid.cpp:269-284), read by uTplot.py / uTerr.py by splitting on
tabs.  The fixture tests/golden/uT_N32.txt holds the reference's own result
(e2e_N32.npz) in that format; the GPU test (test_gpu_driver.py) requires the
./multigrid driver to write exactly these bytes.
"""
import os
import sys

import numpy as np
from conftest import GOLDEN, load_golden

sys.path.insert(0, GOLDEN)
from make_uT_fixture import format_uT  # noqa: E402


def test_uT_fixture_is_reference_result_in_reference_format():
    g = load_golden("e2e_N32.npz")
    with open(os.path.join(GOLDEN, "uT_N32.txt")) as f:
        text = f.read()
    assert text == format_uT(g["uT"], 32)
    lines = text.splitlines()
    assert len(lines) == 33 * 33
    # parsed the way uTplot.py / uTerr.py parse it
    parsed = [l.split("\t") for l in lines]
    assert all(len(p) == 3 for p in parsed)
    ij = [(int(p[0]), int(p[1])) for p in parsed]
    assert ij == [(i, j) for i in range(33) for j in range(33)]
    vals = np.array([float(p[2]) for p in parsed])
    assert np.max(np.abs(vals - g["uT"])) <= 5e-7   # %f keeps 6 decimals
