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


def test_row_block_writer_matches_the_whole_grid_file(tmp_path):
    """libmgx's writer (mgx_write_uT, host code: no GPU) gives the fixture's
    bytes from the whole grid, and from row blocks appended in rank order --
    how a row-partitioned run writes uT.txt without any rank holding the grid
    (multigrid.cpp:269-284).  Ragged blocks, an empty block, odd thread counts."""
    from hpcclassmultigridproject_amd import write_uT
    g = load_golden("e2e_N32.npz")
    u = np.ascontiguousarray(g["uT"], dtype=np.float64)
    with open(os.path.join(GOLDEN, "uT_N32.txt"), "rb") as f:
        want = f.read()
    whole = tmp_path / "whole.txt"
    write_uT(whole, u, 32, nthreads=3)
    assert whole.read_bytes() == want
    W = 33
    blocks = tmp_path / "blocks.txt"
    edges = [0, 8, 8, 16, 24, 33]   # the last block owns the boundary row N
    for k, (a, b) in enumerate(zip(edges[:-1], edges[1:])):
        write_uT(blocks, u[a * W:b * W].copy(), 32, a, b, append=k > 0, nthreads=k + 1)
    assert blocks.read_bytes() == want
    # values %f cannot hold in a short line (the reference blow-up case, K7)
    big = np.full(W * W, -1.7e300)
    write_uT(tmp_path / "big.txt", big, 32, nthreads=2)
    first = (tmp_path / "big.txt").read_text().split("\n", 1)[0]
    assert first == "0\t0\t%f" % -1.7e300
