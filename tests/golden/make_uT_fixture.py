"""Write tests/golden/uT_N32.txt: the reference's own 100-step result at N=32
(e2e_N32.npz, produced by the reference build in make_golden.py) in the
reference's text format, multigrid.cpp:269-284: "%d\t%d\t%f\n", i outer, j inner.
    python tests/golden/make_uT_fixture.py"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def format_uT(u, N):
    u = u.reshape(N + 1, N + 1)
    return "".join("%d\t%d\t%f\n" % (i, j, u[i, j]) for i in range(N + 1) for j in range(N + 1))


if __name__ == "__main__":
    with np.load(os.path.join(HERE, "e2e_N32.npz"), allow_pickle=False) as z:
        text = format_uT(z["uT"], 32)
    with open(os.path.join(HERE, "uT_N32.txt"), "w") as f:
        f.write(text)
