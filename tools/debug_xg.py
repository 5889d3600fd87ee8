"""Where does the cross pass's XG form differ from the separate-strip form?
    python tools/debug_xg.py [N] [L] [cycles]"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from hpcclassmultigridproject_amd import Multigrid, _lib, init_problem  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
L = int(sys.argv[2]) if len(sys.argv) > 2 else 3
C = int(sys.argv[3]) if len(sys.argv) > 3 else 1
u0, v1, v2 = init_problem(N, nthreads=16)
out = {}
for xg in (0, 1):
    _lib.set_tuning("xgroup", xg)
    with Multigrid(N, L, 1.0 / N / 10, -4e-4, device=0) as mg:
        mg.upload(u0, v1, v2)
        mg.rhs()
        norms = [mg.run_cycles(1) for _ in range(C)]
        out[xg] = (mg.download(), norms)
a, b = out[0][0].reshape(N + 1, N + 1), out[1][0].reshape(N + 1, N + 1)
print("norms", out[0][1], out[1][1])
d = a != b
print("differ:", int(d.sum()), "of", d.size)
if d.any():
    rows = np.where(d.any(axis=1))[0]
    cols = np.where(d.any(axis=0))[0]
    print("rows", rows.min(), rows.max(), len(rows))
    print("cols", cols.min(), cols.max(), len(cols))
    print("first cols", cols[:40])
    print("last cols", cols[-20:])
    print("first rows", rows[:20], "last rows", rows[-20:])
    xl = (N + 14 - 512) & ~1
    print("cols rel. group lanes (col-2) % 484 % 128:", np.unique((cols - 2) % 484 % 128)[:80])
    print("hist (col-2)%484:", np.unique((cols - 2) % 484)[:80])
    WG = 484
    print("cols - 16 mod 484 hist", np.bincount((cols - 16) % WG, minlength=WG).nonzero()[0][:60])
    print("cols mod 128 (rel. group origin-14)", np.unique(((cols - 2) % WG) % 128)[:60])
    r = rows[len(rows) // 2]
    print("row", r, "cols", np.where(d[r])[0][:40])
