"""Multi-process (world_size 2 and 4, gloo, CPU) tests of the partitioned path.

* the unique-id broadcast that bootstraps libmgx's RCCL communicator;
* the partition plan from libmgx (mgx_partition) as every rank sees it:
  blocks tile each level, start at even rows, hold >= the ghost width;
* the partitioned V-cycle's data movement (tests/dist_sim.py: libmgx's own
  exchange plan -- the ncclSend/ncclRecv entries its RCCL transport posts --
  executed as gloo send/recv between the processes, libmgx's all-gather rows,
  norm all-reduce) with the oracle's stencils and NaN-poisoned non-local
  rows: each rank's owned rows after two V-cycles are BITWISE the
  single-process oracle's, and the all-reduced norm matches to 1e-12;
* the same for the cross-cycle schedule (one 16-row ghost exchange per cycle
  on level 0; 14 rows pass, 12 fail -- the pass's cone).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

NU = -4e-4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, N, L, nsmooth, min_rows, q, cross=False):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dist_sim import K_GHOST, PartitionedVCycle
        from hpcclassmultigridproject_amd import _lib
        from hpcclassmultigridproject_amd import dist as mgd
        from oracle import oracle as O

        out = {}
        # 1. id broadcast (the bytes libmgx's ncclCommInitRank receives)
        payload = bytes((7 * i + 3) % 256 for i in range(_lib.UNIQUE_ID_BYTES))
        out["id"] = mgd.broadcast_bytes(payload if rank == 0 else None,
                                        _lib.UNIQUE_ID_BYTES) == payload
        # 2. the plan every rank computes
        _lib.set_tuning("dist_min_rows", min_rows)
        plans = [[mgd.partition(N, L, world, r, l) for l in range(L)] for r in range(world)]
        mine = [None] * world
        dist.all_gather_object(mine, [mgd.partition(N, L, world, rank, l) for l in range(L)])
        out["plan_agrees"] = mine == plans
        out["plans"] = plans
        # 3. partitioned V-cycles vs the single-process oracle
        u0, v1, v2 = O.init_problem(N)
        dt = 1.0 / N / 10
        tower = O.Tower(u0, v1, v2, N, L)
        sim = PartitionedVCycle(rank, world, N, L, tower, dt, NU, nsmooth,
                                lambda l: mgd.partition(N, L, world, rank, l),
                                lambda l: mgd.exchange_plan(N, L, world, rank, l),
                                lambda: mgd.gather_plan(N, L, world, rank))
        sim.u[0][:] = u0
        sim.rhs[0] = O.compute_rhs(u0, N, v1, v2, dt, NU, 1.0 / N)
        ncyc = 3 if cross else 2
        norms = [sim.vcycle_cross() if cross else sim.vcycle() for _ in range(ncyc)]
        O.compute_rhs(tower.ufine, N, v1, v2, dt, NU, 1.0 / N, rhs=tower.rhsfine)
        ref_norms = []
        for _ in range(ncyc):
            tower.mg_inner(dt, NU, nsmooth=nsmooth)
            res = O.residual(tower.ufine, tower.rhsfine, N, v1, v2, dt, NU, 1.0 / N)
            ref_norms.append(O.compute_norm(res, N))
        ra, rb, la = mgd.partition(N, L, world, rank, 0)
        ref_rows = tower.ufine.reshape(N + 1, N + 1)[ra:rb]
        got = sim.u_post if cross else sim.owned(sim.u[0])
        out.update(la=la, bitwise=bool(np.array_equal(got, ref_rows)),
                   finite=bool(np.isfinite(got).all()), norms=norms, ref_norms=ref_norms,
                   coarse_iters=sim.coarse_iters, ghost=K_GHOST)
        tower.close()
        q.put((rank, out))
    except Exception as e:   # report, never hang the parent
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


def _run(world, N, L, nsmooth=3, min_rows=16, cross=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, N, L, nsmooth, min_rows, q, cross))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in res[r], res[r]
    return res


@pytest.mark.parametrize("world,N,L,min_rows", [(2, 128, 4, 16), (2, 256, 5, 16),
                                                (4, 256, 4, 16), (2, 1024, 6, 256),
                                                (2, 1024, 6, 512)])   # la = 1
def test_partitioned_vcycle_gloo(world, N, L, min_rows):
    res = _run(world, N, L, min_rows=min_rows)
    for r in range(world):
        o = res[r]
        assert o["id"] and o["plan_agrees"]
        assert o["finite"], "owned rows read non-local data (NaN poison reached them)"
        assert o["bitwise"]
        np.testing.assert_allclose(o["norms"], o["ref_norms"], rtol=1e-12)
    # the plan: blocks tile every partitioned level, even starts, >= ghost rows
    plans, la = res[0]["plans"], res[0]["la"]
    assert 0 < la <= L - 1
    for l in range(L):
        n = N >> l
        blocks = [plans[r][l][:2] for r in range(world)]
        if l >= la:
            assert all(b == (0, n + 1) for b in blocks)
            continue
        assert blocks[0][0] == 0 and blocks[-1][1] == n + 1
        for (a0, b0), (a1, b1) in zip(blocks, blocks[1:]):
            assert b0 == a1
        for a, b in blocks:
            assert a % 2 == 0 and b - a >= res[0]["ghost"] and b - a >= min_rows


def test_partitioned_vcycle_gloo_nsmooth2():
    res = _run(2, 128, 4, nsmooth=2)
    assert all(res[r]["bitwise"] and res[r]["finite"] for r in range(2))


@pytest.mark.parametrize("world,N,L", [(2, 128, 4), (4, 256, 4)])
def test_partitioned_cross_cycle_gloo(world, N, L):
    """The cross-cycle schedule on row blocks: one 16-row ghost exchange per
    cycle feeds post-smoothing, norm and the next pre-smoothing (dist.hip
    dist_cross); u_post after 3 cycles is bitwise the oracle's."""
    res = _run(world, N, L, cross=True)
    for r in range(world):
        o = res[r]
        assert o["finite"] and o["bitwise"], o
        np.testing.assert_allclose(o["norms"], o["ref_norms"], rtol=1e-12)
