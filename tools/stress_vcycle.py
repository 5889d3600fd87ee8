"""Repeat V-cycles for many configs in one process and compare with the CPU checker."""
import sys, hashlib
sys.path.insert(0, '.')
import numpy as np
import hpcclassmultigridproject_amd as pkg
from oracle import oracle as O
O.set_threads(16)
nu = -4e-4
cfgs = [(4096, 3), (1024, 6), (2048, 4), (4096, 5), (8192, 3), (512, 4), (4096, 3)]
bad = 0
for N, L in cfgs:
    dt = 1.0 / N / 10
    u0, v1, v2 = pkg.init_problem(N)
    t = O.Tower(u0, v1, v2, N, L)
    O.compute_rhs(t.ufine, N, v1, v2, dt, nu, 1.0 / N, rhs=t.rhsfine)
    t.mg_inner(dt, nu)
    ref = t.ufine.copy(); t.close()
    for sm, fu in [(0, 3), (0, 2), (0, 1), (2, 3), (1, 3)]:
        for rep in range(3):
            with pkg.Multigrid(N, L, dt, nu, smoother=sm, fuse=fu, device=0) as mg:
                mg.upload(u0, v1, v2); mg.rhs(); mg.mg_inner()
                got = mg.download()
                its = mg.coarse_iterations()
            nbad = int((got != ref).sum())
            if nbad:
                bad += 1
                d = np.argwhere(got.reshape(N+1, N+1) != ref.reshape(N+1, N+1))
                print(f"MISMATCH N={N} L={L} sm={sm} fu={fu} rep={rep} count={nbad} its={its} first={d[:4].tolist()} rows={np.unique(d[:,0])[:20].tolist()}", flush=True)
            else:
                print(f"ok N={N} L={L} sm={sm} fu={fu} rep={rep} its={its}", flush=True)
print("BAD", bad)
