"""A/B of upload-time tuning keys: one context per setting, interleaved timed
rounds in one process, u bitwise equal, per-level device time.
    python tools/ab_keys.py "sep_velocity=1,zero_rows=1" "sep_velocity=1,zero_rows=0" [--N 16384 --L 9 --rounds 3]
"""
import argparse
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from hpcclassmultigridproject_amd import Multigrid, _lib, init_problem  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("settings", nargs="+")
ap.add_argument("--N", type=int, default=16384)
ap.add_argument("--L", type=int, default=9)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--cycles", type=int, default=10)
a = ap.parse_args()
N, L = a.N, a.L
dt, nu = 1.0 / N / 10, -4e-4
u0, v1, v2 = init_problem(N, nthreads=16)
ctx = []
for st in a.settings:
    kv = dict(x.split("=") for x in st.split(",") if x)
    old = {k: _lib.get_tuning(k) for k in kv}
    for k, v in kv.items():
        _lib.set_tuning(k, int(v))
    mg = Multigrid(N, L, dt, nu, device=0)
    mg.upload(u0, v1, v2)
    for k, v in old.items():
        _lib.set_tuning(k, v)
    mg.rhs()
    mg.run_cycles(2)
    ctx.append((st, kv, mg))
times = {st: [] for st, _, _ in ctx}
for r in range(a.rounds):
    for st, kv, mg in ctx:
        old = {k: _lib.get_tuning(k) for k in kv}
        for k, v in kv.items():
            _lib.set_tuning(k, int(v))
        mg.synchronize()
        t0 = time.perf_counter()
        mg.run_cycles(a.cycles)
        mg.synchronize()
        times[st].append((time.perf_counter() - t0) / a.cycles * 1e3)
        for k, v in old.items():
            _lib.set_tuning(k, v)
for st, kv, mg in ctx:
    old = {k: _lib.get_tuning(k) for k in kv}
    for k, v in kv.items():   # launch-time keys apply to the profiled cycles too
        _lib.set_tuning(k, int(v))
    mg.profile_reset()
    mg.profile(True)
    mg.run_cycles(3)
    for k, v in old.items():
        _lib.set_tuning(k, v)
    lv = []
    for l in range(L):
        tot = 0.0
        for k in _lib.KERNEL_NAMES:
            n, ms, b, cb = mg.profile_get_ex(k, l)
            tot += ms
        lv.append(round(tot / 3, 4))
    mg.profile(False)
    print(f"{st:40s} ms/cycle {['%.3f' % x for x in times[st]]}  per level {lv}", flush=True)
ref = ctx[0][2].download()
for st, kv, mg in ctx[1:]:
    print(st, "bitwise vs first:", bool(np.array_equal(mg.download(), ref)), flush=True)
for _, _, mg in ctx:
    mg.close()
