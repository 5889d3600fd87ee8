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
