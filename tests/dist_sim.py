"""CPU model of the row-partitioned V-cycle (dist.hip), for gloo tests.

Test infrastructure: every rank holds each partitioned level as a full-size
array of which only its allocated rows [lo, hi] (owned rows + kGhost ghost
rows, as in dist.hip) are meaningful; every other row is POISONED with NaN
before each smoothing pass, so any dependence on data the rank does not hold
shows up as NaN in its owned rows.  The stencil arithmetic is the oracle's
(oracle/mg_oracle.c, the reference's term order), the data movement is what
dist.hip does, over torch.distributed (gloo): ghost rows from rank +-1
(isend/irecv), all-gather of the restricted rhs into the first replicated
level, all-reduce of the residual's sum of squares.  The partition, the
ghost-row exchange plan and the all-gather rows all come from libmgx itself
(mgx_partition, mgx_exchange_plan, mgx_gather_plan: the entries its RCCL
transport posts as ncclSend/ncclRecv and ncclAllGather), so the processes
here exchange exactly the rows, offsets and counts the RCCL ranks do; a rank's
allocated rows are what that plan receives, everything else is NaN.

Mirrors: dist.hip dist_level (pre pass + restrict, recurse / gather, post
pass + prolong), multigrid.cpp:17-92 for the replicated levels.  Post passes
are communication-avoiding (dist.hip post_ca): a coarse level's corrected u
is NOT exchanged; only its rows within POST_EXT of its block (which its own
post pass computed) are kept, every other row is poisoned before the finer
level prolongs from it.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.distributed as dist

from oracle import oracle as O

K_GHOST = 16        # plan.h kGhost (the fewest ghost rows a block may hold)
POST_EXT = 10       # plan.h kPostExt: rows past its block a coarse post pass computes


class Block:
    def __init__(self, n, ra, rb, xfers=()):
        """Owned rows [ra, rb); allocated rows = owned + what `xfers` (the
        library's exchange plan for this rank) receives."""
        self.n, self.ra, self.rb, self.xfers = n, ra, rb, list(xfers)
        self.lo, self.hi = ra, rb - 1
        for peer, s0, sn, r0, rn in self.xfers:
            assert r0 + rn <= ra or r0 >= rb, "plan receives into owned rows"
            self.lo, self.hi = min(self.lo, r0), max(self.hi, r0 + rn - 1)

    def rows(self, a):
        return a.reshape(self.n + 1, self.n + 1)

    def poison(self, a):
        m = self.rows(a)
        m[: self.lo] = np.nan
        m[self.hi + 1:] = np.nan


def exchange(blk, a, rank, world):
    """The library's exchange plan for this rank and level, posted as gloo
    isend/irecv pairs (dist.hip exchange_rows: ncclSend/ncclRecv)."""
    m = blk.rows(a)
    reqs, recv = [], []
    for peer, s0, sn, r0, rn in blk.xfers:
        reqs.append(dist.isend(torch.from_numpy(m[s0:s0 + sn].copy()), peer))
        buf = torch.empty((rn, blk.n + 1), dtype=torch.float64)
        reqs.append(dist.irecv(buf, peer))
        recv.append((r0, buf))
    for r in reqs:
        r.wait()
    for r0, buf in recv:
        m[r0:r0 + buf.shape[0]] = buf.numpy()


class PartitionedVCycle:
    def __init__(self, rank, world, N, L, tower, dt, nu, nsmooth, plan, xplan, gplan):
        """plan(level) -> (ra, rb, la): mgx_partition for this rank;
        xplan(level) -> mgx_exchange_plan entries; gplan() -> mgx_gather_plan."""
        self.rank, self.world, self.N, self.L = rank, world, N, L
        self.dt, self.nu, self.nsmooth = dt, nu, nsmooth
        self.la = plan(0)[2]
        self.gplan = gplan
        self.blk = [Block(N >> l, *plan(l)[:2], xplan(l)) for l in range(self.la)]
        self.spec = False   # cross-cycle mode: next cycle's pre-smoothing already done
        self.v1 = [tower.level("v1", l) for l in range(L)]
        self.v2 = [tower.level("v2", l) for l in range(L)]
        self.u = [np.zeros((N >> l) ** 2 + 2 * (N >> l) + 1) for l in range(L)]
        self.rhs = [np.zeros_like(x) for x in self.u]
        self.coarse_iters = 0

    def h(self, l):
        return (1.0 / self.N) * 2 ** l

    def _gs(self, l):
        n = self.N >> l
        for _ in range(self.nsmooth):
            O.gauss_seidel(self.u[l], self.rhs[l], n, self.v1[l], self.v2[l], self.dt, self.nu,
                           self.h(l))

    def _res(self, l):
        n = self.N >> l
        return O.residual(self.u[l], self.rhs[l], n, self.v1[l], self.v2[l], self.dt, self.nu,
                          self.h(l))

    # -- replicated levels (multigrid.cpp:17-92 on whole arrays)
    def _full(self, l):
        n = self.N >> l
        if l == self.L - 1:
            res, i = 1.0, 0
            while i < 1000 and res > 1e-5:
                O.gauss_seidel(self.u[l], self.rhs[l], n, self.v1[l], self.v2[l], self.dt,
                               self.nu, self.h(l))
                res = O.compute_norm(self._res(l), n)
                i += 1
            self.coarse_iters += i
            return
        self._gs(l)
        self.rhs[l + 1] = O.restriction(self._res(l), n)
        self.u[l + 1][:] = 0.0
        self._full(l + 1)
        self.u[l] += O.prolongation(self.u[l + 1], n // 2)
        self._gs(l)

    # -- partitioned levels (dist.hip dist_level)
    def _level(self, l, zero, want_norm):
        n, b = self.N >> l, self.blk[l]
        # pre-smoothing pass (+ residual restricted to the coarse rhs)
        if zero:
            self.u[l][:] = 0.0
        else:
            exchange(b, self.u[l], self.rank, self.world)
        b.poison(self.u[l])
        b.poison(self.rhs[l])
        self._gs(l)
        res = self._res(l)
        crs = O.restriction(res, n)   # coarse rows I <- fine rows 2I
        nc = n // 2
        c = crs.reshape(nc + 1, nc + 1)
        tgt = self.rhs[l + 1].reshape(nc + 1, nc + 1)
        own = slice((b.ra + 1) // 2, (b.rb + 1) // 2)   # I with 2I in [ra, rb)
        tgt[own] = c[own]
        if l + 1 < self.la:
            exchange(self.blk[l + 1], self.rhs[l + 1], self.rank, self.world)
            self._level(l + 1, True, False)
        else:
            self._gather_rhs(l + 1)
            self.u[l + 1][:] = 0.0
            self._full(l + 1)
        # post-smoothing pass: prolongation + add, sweeps (+ residual norm)
        exchange(b, self.u[l], self.rank, self.world)
        if l + 1 < self.la:
            self._keep_post_rows(l + 1)
        b.poison(self.u[l])
        self.u[l] += O.prolongation(self.u[l + 1], nc)
        self._gs(l)
        if want_norm:
            r = self._res(l).reshape(n + 1, n + 1)
            i0, i1 = max(1, b.ra), min(n, b.rb)
            part = torch.tensor([float(np.sum(r[i0:i1, 1:n] ** 2))], dtype=torch.float64)
            dist.all_reduce(part)
            return math.sqrt(float(part[0]))
        return None

    def _keep_post_rows(self, l):
        """Level l's u after its post pass: valid on its block +- POST_EXT rows
        only (no exchange); poison the rest."""
        b = self.blk[l]
        m = b.rows(self.u[l])
        m[: max(0, b.ra - POST_EXT)] = np.nan
        m[b.rb + POST_EXT:] = np.nan

    def _gather_rhs(self, l):
        """dist.hip gather_rhs: the in-place all-gather of mgx_gather_plan's rows."""
        n = self.N >> l
        la, r0, q = self.gplan()
        assert la == l
        m = self.rhs[l].reshape(n + 1, n + 1)
        mine = torch.from_numpy(m[r0:r0 + q].copy())
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(parts, mine)
        for r, t in enumerate(parts):
            m[r * q:(r + 1) * q] = t.numpy()   # rank-major (ncclAllGather in place)

    def _restrict_owned(self, l):
        """Residual of level l restricted into the owned rows of rhs[l+1]."""
        n, b = self.N >> l, self.blk[l]
        nc = n // 2
        crs = O.restriction(self._res(l), n).reshape(nc + 1, nc + 1)
        tgt = self.rhs[l + 1].reshape(nc + 1, nc + 1)
        own = slice((b.ra + 1) // 2, (b.rb + 1) // 2)
        tgt[own] = crs[own]

    def _coarse_ready(self, l):
        if l + 1 < self.la:
            exchange(self.blk[l + 1], self.rhs[l + 1], self.rank, self.world)
            return
        self._gather_rhs(l + 1)

    def _coarse_cycle(self, l):
        if l < self.la:
            self._level(l, True, False)
        else:
            self.u[l][:] = 0.0
            self._full(l)

    def vcycle_cross(self):
        """dist.hip dist_vcycle with the cross-cycle pass on level 0: ONE u
        ghost exchange (16 rows) feeds prolongation + post-smoothing + norm +
        the next cycle's pre-smoothing + restriction."""
        n, b = self.N, self.blk[0]
        if not self.spec:   # first cycle: plain pre-smoothing pass
            exchange(b, self.u[0], self.rank, self.world)
            b.poison(self.u[0])
            b.poison(self.rhs[0])
            self._gs(0)
            self._restrict_owned(0)
            self._coarse_ready(0)
        self._coarse_cycle(1)
        exchange(b, self.u[0], self.rank, self.world)
        if 1 < self.la:
            self._keep_post_rows(1)
        b.poison(self.u[0])
        b.poison(self.rhs[0])
        self.u[0] += O.prolongation(self.u[1], n // 2)
        self._gs(0)   # post-smoothing of this cycle
        r = self._res(0).reshape(n + 1, n + 1)
        i0, i1 = max(1, b.ra), min(n, b.rb)
        part = torch.tensor([float(np.sum(r[i0:i1, 1:n] ** 2))], dtype=torch.float64)
        dist.all_reduce(part)
        self.u_post = self.owned(self.u[0]).copy()
        self._gs(0)   # the next cycle's pre-smoothing, no exchange in between
        self._restrict_owned(0)
        self._coarse_ready(0)
        self.spec = True
        return math.sqrt(float(part[0]))

    def vcycle(self):
        """One V-cycle from u[0], rhs[0]; returns the all-reduced residual norm."""
        if self.la == 0:
            self._full(0)
            return O.compute_norm(self._res(0), self.N)
        return self._level(0, False, True)

    def owned(self, a, l=0):
        b = self.blk[l] if l < self.la else Block(self.N >> l, 0, (self.N >> l) + 1)
        return b.rows(a)[b.ra:b.rb]
