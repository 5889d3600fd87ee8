"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only where /root/reference exists (this container): oracle/Makefile
compiles the unmodified reference sources into oracle/_ref/libmgref.so and this
script calls the reference's own gauss_seidel / residual / compute_norm /
prolongation / restriction / compute_rhs / mg_inner / timestepper through the
C harness (oracle/ref_harness.cpp).  Only inputs and outputs are written
(numpy .npz without pickles, JSON); nothing of the reference's source text.

    python tests/golden/make_golden.py [--large]

--large adds the N=16384 fixtures (one reference V-cycle, and 2 timesteps
with OMP threads; several minutes).
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

SEED = 20220501
NU = -4e-4               # multigrid.cpp:235
D, LNG, I = C.c_double, C.c_long, C.c_int


def p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def stats(u, N):
    u2 = u.reshape(N + 1, N + 1)
    i = int(np.argmax(u))
    return {"N": N, "sum": repr(float(u.sum())), "sumsq": repr(float((u * u).sum())),
            "max": repr(float(u.max())), "argmax": [i // (N + 1), i % (N + 1)],
            "center": repr(float(u2[N // 2, N // 2])),
            "sha256": hashlib.sha256(u.tobytes()).hexdigest()}


def strided(u, N, count=65):
    step = max(1, N // (count - 1))
    return u.reshape(N + 1, N + 1)[::step, ::step].copy()


def ops_fixture(N):
    R = O.ref()
    rng = np.random.default_rng(SEED + N)
    cnt = (N + 1) ** 2
    _, v1, v2 = O.init_problem(N)
    u = rng.uniform(-1.0, 1.0, cnt)
    rhs = rng.uniform(-1.0, 1.0, cnt)
    k, h = 1.0 / N / 10, 1.0 / N
    out = {"u": u.copy(), "rhs": rhs.copy(), "v1": v1, "v2": v2,
           "params": np.array([N, k, NU, h])}
    g = u.copy()
    R.ref_gauss_seidel(p(g), p(rhs), LNG(N), p(v1), p(v2), D(k), D(NU), D(h), I(1))
    out["gs"] = g
    res = np.zeros(cnt)
    R.ref_residual(p(res), p(u), p(rhs), LNG(N), p(v1), p(v2), D(k), D(NU), D(h))
    out["res"] = res
    out["norm"] = np.array([R.ref_compute_norm(p(res), LNG(N))])
    cr = np.zeros(cnt)
    R.ref_compute_rhs(p(cr), p(u), LNG(N), p(v1), p(v2), D(k), D(NU), D(h))
    out["crhs"] = cr
    up = np.zeros((2 * N + 1) ** 2)
    R.ref_prolongation(p(up), p(u), I(N))
    out["prol"] = up
    rs = np.zeros((N // 2 + 1) ** 2)
    R.ref_restriction(p(rs), p(u), I(N))
    out["restr"] = rs
    np.savez_compressed(os.path.join(HERE, f"ops_N{N}.npz"), **out)


def e2e_fixture(N, nu, tag, summary):
    maxlvl = int(math.log2(N)) - 4
    u0, v1, v2 = O.init_problem(N)
    dx = 1.0 / N
    dt = dx / 10
    T = 100 * dt
    t = time.time()
    uT = O.ref_timestepper(u0, v1, v2, nu, maxlvl, N, dt, T, dx, 1e-6, 1, nthreads=1)
    # cycles per step: the reference prints nothing, so take them from the
    # restatement after checking it is bitwise equal on this case
    uo, cyc = O.timestepper(u0, v1, v2, nu, maxlvl, N, dt, T, dx)
    assert np.array_equal(uo, uT), f"restatement differs from reference at {tag}"
    np.savez_compressed(os.path.join(HERE, f"e2e_{tag}.npz"), uT=uT,
                        cycles=np.array(cyc, dtype=np.int32),
                        params=np.array([N, maxlvl, nu, dt, T, 1e-6]))
    s = stats(uT, N)
    s.update({"maxlvl": maxlvl, "nu": nu, "steps": int(T / dt), "cycles": sorted(set(cyc)),
              "ref_seconds": round(time.time() - t, 3)})
    summary["e2e"][tag] = s


def vcycle_fixture(N, maxlvl, nthreads, tag, summary, keep_full=False, tower=0):
    """One reference V-cycle; tower 1 = the correct velocity tower, built by
    the reference's own restriction at each level's true size
    (oracle/ref_harness.cpp build, correct = 1)."""
    u0, v1, v2 = O.init_problem(N)
    dt = 1.0 / N / 10
    u = u0.copy()
    t = time.time()
    res = O.ref().ref_vcycle_once_tower(p(u), p(v1), p(v2), I(N), I(maxlvl), D(dt), D(NU),
                                        I(1), I(nthreads), I(tower))
    s = stats(u, N)
    s.update({"maxlvl": maxlvl, "nsmooth": 3, "res_after": repr(res), "nthreads": nthreads,
              "tower": "correct" if tower else "reference",
              "ref_seconds": round(time.time() - t, 2)})
    summary["vcycle"][tag] = s
    data = {"sample": strided(u, N), "params": np.array([N, maxlvl, NU, dt])}
    if keep_full:
        data["u"] = u
    np.savez_compressed(os.path.join(HERE, f"vcycle_{tag}.npz"), **data)


def correct_tower_fixtures(summary, large=True):
    """The correct velocity tower (every level injected from the one above at
    its true size) through the reference's own restriction and mg_inner: one
    V-cycle at N=4096, L=7 and (large) at the headline size N=16384, L=9."""
    vcycle_fixture(4096, 7, 8, "N4096_L7_correct", summary, tower=1)
    if large:
        vcycle_fixture(16384, 9, 8, "N16384_L9_correct", summary, tower=1)


def config2_fixture(summary, nthreads=8):
    """BASELINE configs[1]: N=4096, 3-level V-cycle, 2 pre/post RB-GS sweeps,
    from the reference built with NITER=2 (oracle/Makefile libmgref_nu2.so):
    one V-cycle and two timesteps (sha256 + stats, cycles per step)."""
    N, maxlvl = 4096, 3
    u0, v1, v2 = O.init_problem(N)
    dx = 1.0 / N
    dt = dx / 10
    u = u0.copy()
    t = time.time()
    res = O.ref(2).ref_vcycle_once(p(u), p(v1), p(v2), I(N), I(maxlvl), D(dt), D(NU), I(1),
                                   I(nthreads))
    s = stats(u, N)
    s.update({"maxlvl": maxlvl, "nsmooth": 2, "res_after": repr(res), "nthreads": nthreads,
              "ref_seconds": round(time.time() - t, 2)})
    summary["vcycle"]["N4096_L3_nu2"] = s
    steps = 2
    t = time.time()
    uT = O.ref_timestepper(u0, v1, v2, NU, maxlvl, N, dt, steps * dt, dx, 1e-6, 1,
                           nthreads=nthreads, nsmooth=2)
    secs = time.time() - t
    O.set_threads(nthreads)
    uo, cyc = O.timestepper(u0, v1, v2, NU, maxlvl, N, dt, steps * dt, dx, nsmooth=2)
    assert np.array_equal(uo, uT), "restatement differs from the NITER=2 reference"
    s = stats(uT, N)
    s.update({"maxlvl": maxlvl, "nsmooth": 2, "steps": steps, "cycles": list(cyc),
              "nthreads": nthreads, "ref_seconds": round(secs, 1)})
    summary["steps"]["N4096_L3_nu2_2steps"] = s


def large_steps(N, maxlvl, steps, nthreads, summary):
    u0, v1, v2 = O.init_problem(N)
    dx = 1.0 / N
    dt = dx / 10
    t = time.time()
    uT = O.ref_timestepper(u0, v1, v2, NU, maxlvl, N, dt, steps * dt, dx, 1e-6, 1,
                           nthreads=nthreads)
    s = stats(uT, N)
    s.update({"maxlvl": maxlvl, "steps": steps, "nthreads": nthreads,
              "ref_seconds": round(time.time() - t, 1)})
    summary["steps"][f"N{N}_L{maxlvl}_{steps}steps"] = s
    np.savez_compressed(os.path.join(HERE, f"steps_N{N}.npz"), sample=strided(uT, N),
                        params=np.array([N, maxlvl, NU, dt, steps]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", action="store_true")
    ap.add_argument("--only-config2", action="store_true",
                    help="add the config-2 (NITER=2) fixtures to summary.json and stop")
    ap.add_argument("--only-correct-tower", action="store_true",
                    help="add the correct-tower V-cycle fixtures (N=4096 L=7 and N=16384 "
                         "L=9) to summary.json and stop")
    args = ap.parse_args()
    if not O.ref_available():
        sys.exit("oracle/_ref/libmgref.so missing: build with `make -C oracle` here")
    path = os.path.join(HERE, "summary.json")
    summary = json.load(open(path)) if os.path.exists(path) else {}
    summary.setdefault("e2e", {})
    summary.setdefault("vcycle", {})
    summary.setdefault("steps", {})
    summary["generator"] = "tests/golden/make_golden.py (reference compiled by oracle/Makefile)"
    if args.only_config2 or args.only_correct_tower:
        if args.only_config2:
            config2_fixture(summary)
        else:
            correct_tower_fixtures(summary)
        with open(path, "w") as f:
            json.dump(summary, f, indent=1, sort_keys=True)
        return
    for N in (8, 16, 32, 64):
        ops_fixture(N)
    for N, nu, tag in ((32, NU, "N32"), (64, NU, "N64"), (128, NU, "N128"),
                       (128, -0.01, "N128_nu001")):
        e2e_fixture(N, nu, tag, summary)
    vcycle_fixture(256, 4, 1, "N256_L4", summary, keep_full=True)
    vcycle_fixture(1024, 6, 8, "N1024_L6", summary)
    vcycle_fixture(4096, 3, 8, "N4096_L3", summary)
    config2_fixture(summary)
    correct_tower_fixtures(summary, large=args.large)
    if args.large:
        vcycle_fixture(16384, 9, 8, "N16384_L9", summary)
        large_steps(16384, 9, 2, 8, summary)
    with open(path, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1)[:3000])


if __name__ == "__main__":
    main()
