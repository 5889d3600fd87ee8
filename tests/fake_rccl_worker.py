"""TEST INFRASTRUCTURE: libmgx's RCCL branch with peers on ONE GPU.

Run by tests/test_gpu_fake_rccl.py as one child process with
MGX_LIB=tests/fake_rccl/libmgx_fakerccl.so: libmgx's own objects linked against
the in-process fake RCCL of tests/fake_rccl/fake_rccl.hip, so `mgx_create_dist`
and everything after it take the RCCL code path of dist.hip (ncclSend/Recv
ghost exchanges, the in-place all-gathers, the norm all-reduce, the download's
all-gather + broadcast, the overlapped exchange on the second stream) with
`world` peers that are threads of this process on device 0.

Per scenario every rank runs the same sequence as a one-GPU context (the
oracle of this test is the single-GPU solver, itself pinned bitwise to the
reference at these sizes by tests/test_gpu_solver.py): upload (whole grid or
row blocks), compute_rhs, 2 cycles of mg_outer's pattern, 2 time steps, one
plain V-cycle; u is compared BITWISE after each phase (each rank's owned rows,
and the whole grid where the scenario downloads it), norms to 1e-11, cycle
counts exactly.  The anchor for what the transport carries is the reference's
single-stream solver, /root/reference/multigrid.cu:51-92 (it has no
communication of its own).

usage: fake_rccl_worker.py SCENARIOS_JSON OUT_JSON
"""
import ctypes as C
import json
import os
import sys
import threading
import time
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
assert os.environ.get("MGX_LIB", "").endswith("libmgx_fakerccl.so"), "run with MGX_LIB set"

from hpcclassmultigridproject_amd import (Multigrid, _lib, init_problem,  # noqa: E402
                                          init_problem_rows)
from hpcclassmultigridproject_amd import dist as D  # noqa: E402

NU = -4e-4
CALLS = ["ncclCommInitRank", "ncclCommSplit", "ncclGroupStart", "ncclGroupEnd", "ncclSend",
         "ncclRecv", "ncclAllGather", "ncclAllReduce", "ncclBroadcast", "ncclCommDestroy"]


def fake():
    f = C.CDLL(_lib.LIB_PATH)   # the same handle libmgx was loaded with
    f.fake_rccl_calls.restype = C.c_long
    f.fake_rccl_calls.argtypes = [C.c_char_p]
    f.fake_rccl_error.restype = C.c_char_p
    f.fake_rccl_bytes.restype = C.c_long
    f.fake_rccl_thread_calls.restype = C.c_long
    f.fake_rccl_thread_calls.argtypes = [C.c_char_p]
    f.fake_rccl_order_violations.restype = C.c_long
    f.fake_rccl_order_message.restype = C.c_char_p
    f.fake_rccl_rank_idle.restype = C.c_int
    return f


def sequence(mg, full_download, upload, calls=None):
    """The calls every rank (and the one-GPU context) makes; -> results.
    Per phase: the cross-pass launches (K_XSMOOTH events of this context) and,
    when `calls` is given (a rank), the NCCL calls this rank made in it."""
    out = {"phase_xsmooth": {}, "phase_calls": {}, "idle_after_sync": []}
    upload(mg)
    mg.profile(True, finest_only=True)

    def phase(name, fn):
        mg.synchronize()
        c0 = calls() if calls else None
        mg.profile_reset()
        r = fn()
        mg.synchronize()
        if calls:   # mgx_synchronize left no RCCL operation of this rank in flight
            out["idle_after_sync"].append(bool(_FAKE.fake_rccl_rank_idle()))
        out["phase_xsmooth"][name] = mg.profile_get(_lib.K_XSMOOTH, 0)[0]
        if calls:
            c1 = calls()
            out["phase_calls"][name] = {k: c1[k] - c0[k] for k in c1}
        return r

    phase("rhs", mg.rhs)
    out["norms"] = [phase(f"cycle{i}", lambda: mg.run_cycles(1)) for i in range(2)]
    out["u_cycles"] = mg.download_rows(0)
    if full_download:
        out["u_full"] = mg.download()
    out["steps"] = [phase(f"step{i}", mg.step) for i in range(2)]
    out["u_steps"] = mg.download_rows(0)
    # no norm: the plain partitioned V-cycle on every level
    phase("vcycle", mg.mg_inner)
    out["u_vcycle"] = mg.download_rows(0)
    out["xsmooth"] = sum(out["phase_xsmooth"].values())
    out["rows"] = mg.owned_rows(0)
    return out


def run_scenario(sc, ref_cache):
    N, L, G = sc["N"], sc["L"], sc["world"]
    tower = _lib.TOWER_CORRECT if sc.get("row_upload") else _lib.TOWER_REFERENCE
    dt = 1.0 / N / 10
    _lib.set_tuning("dist_min_rows", sc.get("min_rows", 256))
    _lib.set_tuning("dist_overlap", sc.get("overlap", 0))
    # test hook: 0 drops dist.hip's RCCL operation chain (the negative case of
    # the fake's happens-before check)
    _lib.set_tuning("dist_comm_chain", sc.get("comm_chain", 1))
    fp = _lib.FP_FMA if sc.get("fp") == "fma" else _lib.FP_BITWISE
    u0, v1, v2 = init_problem(N)
    key = (N, L, tower, fp)
    if key not in ref_cache:
        # (step_cross off: its time-step cross pass is single-GPU only, so with
        # it the one-GPU context's steps would launch one cross pass more than
        # the partitioned ones; the results are bitwise the same either way)
        old_sc = _lib.get_tuning("step_cross")
        try:
            _lib.set_tuning("step_cross", 0)
            with Multigrid(N, L, dt, NU, device=0, tower_mode=tower, fp_mode=fp) as mg:
                ref_cache[key] = sequence(mg, True, lambda m: m.upload(u0, v1, v2))
        finally:
            _lib.set_tuning("step_cross", old_sc)
    ref = ref_cache[key]
    full = sc.get("full_download", False)
    uid = D.unique_id()
    res, errs = [None] * G, [None] * G
    upload_lock = threading.Lock()   # whole-grid uploads build a full tower each

    def rank_main(r):
        try:
            def upload(m):
                if sc.get("row_upload"):
                    lo, hi = m.dist_rows(0)
                    m.upload_rows([init_problem_rows(N, lo, hi + 1)])
                else:
                    with upload_lock:
                        m.upload(u0, v1, v2)
            with Multigrid(N, L, dt, NU, device=0, world=G, rank=r, unique_id=uid,
                           tower_mode=tower, fp_mode=fp) as mg:
                out = sequence(mg, full, upload, calls_now)
                out["la"] = mg.dist_info()[2]
            res[r] = out
        except Exception as e:   # noqa: BLE001 -- reported to the test
            errs[r] = f"{type(e).__name__}: {e}\n{traceback.format_exc()}"

    viol0 = _FAKE.fake_rccl_order_violations()
    th = [threading.Thread(target=rank_main, args=(r,), daemon=True) for r in range(G)]
    t0 = time.time()
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    if any(t.is_alive() for t in th):
        # a rank died with peers blocked in a collective: report and bail out
        print(json.dumps({"hung": sc, "errors": errs}), flush=True)
        os._exit(3)
    _lib.set_tuning("dist_comm_chain", 1)
    verdict = {"scenario": sc, "seconds": round(time.time() - t0, 2), "errors": errs,
               "bitwise": {}, "norm_rel_err": 0.0, "steps_equal": True,
               # RCCL operations of a rank issued while its previous one was not
               # ordered before them (fake_rccl.hip happens-before model)
               "order_violations": _FAKE.fake_rccl_order_violations() - viol0,
               "order_message": _FAKE.fake_rccl_order_message().decode()}
    if any(errs):
        return verdict
    W = N + 1
    for phase in ("u_cycles", "u_steps", "u_vcycle"):
        ok = True
        for r in range(G):
            ra, rb = res[r]["rows"]
            ok = ok and res[r][phase].size == (rb - ra) * W and bool(
                np.array_equal(res[r][phase], ref[phase][ra * W:rb * W]))
        verdict["bitwise"][phase] = ok
    if full:
        verdict["bitwise"]["u_full"] = all(bool(np.array_equal(res[r]["u_full"], ref["u_full"]))
                                           for r in range(G))
    for r in range(G):
        e = np.max(np.abs(np.array(res[r]["norms"]) - ref["norms"]) / np.abs(ref["norms"]))
        verdict["norm_rel_err"] = max(verdict["norm_rel_err"], float(e))
        verdict["steps_equal"] = verdict["steps_equal"] and res[r]["steps"] == ref["steps"]
    verdict["cycles_per_step"] = res[0]["steps"]
    verdict["xsmooth_launches"] = [res[r]["xsmooth"] for r in range(G)]
    verdict["ref_xsmooth_launches"] = ref["xsmooth"]
    verdict["phase_xsmooth"] = [res[r]["phase_xsmooth"] for r in range(G)]
    verdict["ref_phase_xsmooth"] = ref["phase_xsmooth"]
    # NCCL calls per phase of every rank (thread-local counters of the fake)
    verdict["phase_calls"] = [res[r]["phase_calls"] for r in range(G)]
    verdict["replicated_level"] = res[0]["la"]
    verdict["idle_after_sync"] = all(all(res[r]["idle_after_sync"]) for r in range(G))
    return verdict


_FAKE = None


def calls_now():
    """NCCL calls made so far by the calling thread (this rank)."""
    return {n: _FAKE.fake_rccl_thread_calls(n.encode()) for n in CALLS}


def main():
    global _FAKE
    scenarios = json.loads(open(sys.argv[1]).read())
    f = _FAKE = fake()
    ref_cache = {}
    out = {"scenarios": []}
    for sc in scenarios:
        v = run_scenario(sc, ref_cache)
        out["scenarios"].append(v)
        print(json.dumps({k: v[k] for k in v if k != "errors"}), flush=True)
    out["calls"] = {n: f.fake_rccl_calls(n.encode()) for n in CALLS}
    out["fake_error"] = f.fake_rccl_error().decode()
    out["bytes"] = f.fake_rccl_bytes()
    with open(sys.argv[2], "w") as fh:
        json.dump(out, fh)


if __name__ == "__main__":
    main()
