"""Multi-GPU plumbing for the row-partitioned solver.

One process per GPU.  libmgx owns the RCCL communicator; torch.distributed
only brokers the 128-byte unique id from rank 0 (any backend, gloo included)
and reads RANK / WORLD_SIZE / LOCAL_RANK.  The partition plan is computed by
libmgx (``mgx_partition``) so that host code and kernels agree on it.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _lib
from ._lib import check, lib


def env_rank():
    """-> (rank, world, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def unique_id() -> bytes:
    """A fresh RCCL unique id (call on ONE rank, share with the others)."""
    buf = C.create_string_buffer(_lib.UNIQUE_ID_BYTES)
    check(lib().mgx_dist_unique_id(buf))
    return buf.raw


def broadcast_bytes(data, nbytes: int, group=None) -> bytes:
    """Broadcast `nbytes` bytes from rank 0 (data is ignored on other ranks)."""
    import torch
    import torch.distributed as dist

    payload = torch.zeros(nbytes, dtype=torch.uint8)
    if dist.get_rank(group) == 0:
        if data is None or len(data) != nbytes:
            raise ValueError(f"rank 0 must supply {nbytes} bytes")
        payload[:] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    if dist.get_backend(group) == "nccl":   # RCCL broadcasts device tensors only
        payload = payload.cuda()
    dist.broadcast(payload, src=0, group=group)
    return bytes(payload.cpu().numpy().tobytes())


def broadcast_unique_id(group=None) -> bytes:
    """Make the RCCL id on rank 0 and broadcast it over torch.distributed."""
    import torch.distributed as dist

    uid = unique_id() if dist.get_rank(group) == 0 else None
    return broadcast_bytes(uid, _lib.UNIQUE_ID_BYTES, group)


def partition(n: int, maxlvl: int, world: int, rank: int, level: int):
    """-> (ra, rb, first_replicated_level): rows [ra, rb) of `level` on `rank`."""
    ra, rb, la = C.c_int(), C.c_int(), C.c_int()
    check(lib().mgx_partition(n, maxlvl, world, rank, level, C.byref(ra), C.byref(rb),
                              C.byref(la)))
    return ra.value, rb.value, la.value


def exchange_plan(n: int, maxlvl: int, world: int, rank: int, level: int):
    """Ghost-row transfers of `rank` on `level` as libmgx executes them (both
    transports): [(peer, send_row, send_rows, recv_row, recv_rows), ...]."""
    cnt = C.c_int()
    buf = (C.c_int * 10)()
    check(lib().mgx_exchange_plan(n, maxlvl, world, rank, level, C.byref(cnt), buf, 2))
    return [tuple(buf[5 * i:5 * i + 5]) for i in range(cnt.value)]


def gather_plan(n: int, maxlvl: int, world: int, rank: int):
    """-> (level, row0, rows): rows `rank` contributes to the all-gather into the
    first replicated level."""
    lv, r0, rows = C.c_int(), C.c_int(), C.c_int()
    check(lib().mgx_gather_plan(n, maxlvl, world, rank, C.byref(lv), C.byref(r0),
                                C.byref(rows)))
    return lv.value, r0.value, rows.value


def rccl_selfcheck(world: int, rank: int, device: int, n: int = 4096, maxlvl: int = 7,
                   cycles: int = 2, group=None, min_rows=(), candidate_fp: str = "fma") -> dict:
    """Run libmgx's RCCL transport with real peers against a single-GPU context.

    Every rank builds a row-partitioned context of the same small problem
    (``dist_min_rows`` 16, so levels 0..5 are split even at world 8; n >= 4096,
    so the finest level runs the cross-cycle pass, asserted by its launch
    count) and runs ``cycles`` V-cycles with it -- ghost send/recv, the
    all-gather into the replicated levels, the norm all-reduce, the
    all-gather + broadcast of the download -- once with the exchanges on the
    compute stream and overlapped (``dist_overlap`` 0 / 1 / 2), in both
    arithmetic modes; rank 0 compares u bitwise and the norms to 1e-11 with a
    one-GPU context of the same fp_mode.  Collective over
    the torch.distributed group (its backend only brokers the unique ids and
    the verdict).  -> {"bitwise": bool, "norm_rel_err": float, "modes": {overlap:
    {...}}, ...} on every rank.

    min_rows: further ``dist_min_rows`` values to check (bench.py's partition
    candidates), each with every overlap mode in the ``candidate_fp`` mode
    only -> "candidates": {"<min_rows>:<overlap>": {...}}; a candidate the
    bench may time has passed here first.
    """
    import numpy as np
    import torch
    import torch.distributed as dist

    from .multigrid import Multigrid, init_problem

    dt, nu = 1.0 / n / 10, -4e-4
    u0, v1, v2 = init_problem(n)
    old_rows, old_ov = _lib.get_tuning("dist_min_rows"), _lib.get_tuning("dist_overlap")
    fps = {"bitwise": _lib.FP_BITWISE, "fma": _lib.FP_FMA}
    ref = {}
    if rank == 0:
        for name, fp in fps.items():
            with Multigrid(n, maxlvl, dt, nu, device=device, fp_mode=fp) as mg:
                mg.upload(u0, v1, v2)
                mg.rhs()
                ref[name] = ([mg.run_cycles(1) for _ in range(cycles)], mg.download())
    # per dist_overlap mode: [bitwise so far (both fp modes), max norm error]
    modes, las = {}, {}
    # (dist_min_rows, overlap, fp modes): 16 in both fp modes (levels 0..5
    # split even at world 8: every exchange of the schedule), then the bench's
    # candidates in its own fp mode
    runs = [(16, ov, tuple(fps)) for ov in (0, 1, 2)]
    runs += [(mr, ov, (candidate_fp,)) for mr in min_rows if mr != 16 for ov in (0, 1, 2)]
    try:
        for mr, ov, names in runs:
            _lib.set_tuning("dist_min_rows", mr)
            _lib.set_tuning("dist_overlap", ov)
            ok, err = True, 0.0
            for name in names:
                fp = fps[name]
                uid = broadcast_unique_id(group)
                with Multigrid(n, maxlvl, dt, nu, device=device, world=world, rank=rank,
                               unique_id=uid, fp_mode=fp) as mg:
                    las[mr] = mg.dist_info()[2]
                    mg.upload(u0, v1, v2)
                    mg.profile(True, finest_only=True)
                    mg.rhs()
                    norms = [mg.run_cycles(1) for _ in range(cycles)]
                    # the cross-cycle pass (and so the overlapped exchange) really ran
                    ok = ok and mg.profile_get(_lib.K_XSMOOTH, 0)[0] > 0
                    u = mg.download()
                if rank == 0:
                    # u bitwise the one-GPU context's of the same fp mode (the
                    # fma forms do not depend on the partition either)
                    ok = ok and bool(np.array_equal(u, ref[name][1]))
                    err = max(err, float(np.max(np.abs(np.array(norms) - ref[name][0]) /
                                                np.abs(ref[name][0]))))
            modes[(mr, ov)] = [ok, err]
    finally:
        _lib.set_tuning("dist_min_rows", old_rows)
        _lib.set_tuning("dist_overlap", old_ov)
    keys = [(mr, ov) for mr, ov, _ in runs]
    verdict = torch.tensor([x for k in keys for x in (1.0 if modes[k][0] else 0.0, modes[k][1])],
                           dtype=torch.float64)
    if dist.get_backend(group) == "nccl":
        verdict = verdict.cuda()
    dist.broadcast(verdict, src=0, group=group)
    v = verdict.cpu().tolist()
    res = {k: {"bitwise": v[2 * i] == 1.0, "norm_rel_err": v[2 * i + 1],
               "passed": v[2 * i] == 1.0 and v[2 * i + 1] <= 1e-11}
           for i, k in enumerate(keys)}
    per = {str(ov): res[(mr, ov)] for mr, ov in keys if mr == 16}
    cand = {f"{mr}:{ov}": dict(res[(mr, ov)], partitioned_levels=las.get(mr))
            for mr, ov in keys if mr != 16}
    return {"N": n, "levels": maxlvl, "cycles": cycles, "partitioned_levels": las.get(16),
            "fp_modes": list(fps), "overlap": [0, 1, 2], "modes": per,
            "candidates": cand, "candidate_fp": candidate_fp,
            "bitwise": all(m["bitwise"] for m in res.values()),
            "norm_rel_err": max(m["norm_rel_err"] for m in res.values()),
            "passed": all(m["passed"] for m in res.values())}
