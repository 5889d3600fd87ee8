"""A/B: the finest cross pass with exact velocity factors (sep_velocity 1) vs
the 2-D v1 / v2 arrays (0), N=16384 L=9: u bitwise equal, ms per V-cycle and
per-kernel finest-level device time, interleaved rounds in one process.
    python tools/ab_sep.py [N] [L] [rounds]
"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from hpcclassmultigridproject_amd import Multigrid, _lib, init_problem  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
L = int(sys.argv[2]) if len(sys.argv) > 2 else 9
R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dt, nu = 1.0 / N / 10, -4e-4
u0, v1, v2 = init_problem(N, nthreads=16)
ctx = {}
for sv in (1, 0):
    _lib.set_tuning("sep_velocity", sv)
    t0 = time.perf_counter()
    mg = Multigrid(N, L, dt, nu, device=0)
    mg.upload(u0, v1, v2)
    import ctypes as C
    fac = C.c_int()
    _lib.check(_lib.lib().mgx_velocity_factored(mg.handle, C.byref(fac)))
    print(f"sep_velocity={sv}: upload {time.perf_counter() - t0:.2f} s, factored={fac.value}",
          flush=True)
    mg.rhs()
    mg.run_cycles(2)
    ctx[sv] = mg
res = {0: [], 1: []}
for r in range(R):
    for sv in (1, 0):
        mg = ctx[sv]
        mg.synchronize()
        t0 = time.perf_counter()
        mg.run_cycles(10)
        mg.synchronize()
        res[sv].append((time.perf_counter() - t0) / 10 * 1e3)
for sv in (1, 0):
    mg = ctx[sv]
    mg.profile_reset()
    mg.profile(True)
    mg.run_cycles(3)
    out = {}
    for k, name in _lib.KERNEL_NAMES.items():
        n, ms, b, cb = mg.profile_get_ex(k, 0)
        if n:
            out[name] = (round(ms / 3, 4), round(cb / n / 1e9, 3), round(cb / (ms * 1e-3) / 1e12, 2))
    mg.profile(False)
    print(f"sep={sv}: ms/cycle {['%.3f' % x for x in res[sv]]}  level0 (ms/cycle, GB/launch, TB/s): {out}",
          flush=True)
a, b = ctx[1].download(), ctx[0].download()
print("bitwise:", bool(np.array_equal(a, b)), flush=True)
for mg in ctx.values():
    mg.close()
