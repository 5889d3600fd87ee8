"""The multi-GPU exchange plan (dist.hip ghost_plan / gather_rows), host only.

Both transports execute ONE plan: RCCL posts each entry as ncclSend(send rows)
+ ncclRecv(recv rows) to its peer; the virtual-rank transport (the one-GPU
parity tests) copies sender rows into the receiver's rows.  Checked here for
every rank of G = 2, 4, 8 (and 16) on every partitioned level, at the sizes
of configs C2-C5:
  * pairing: what rank r sends peer p is exactly what p receives from r (same
    global rows, same count) -- an ncclSend/ncclRecv count mismatch would hang
    or corrupt the real run;
  * sends read only owned rows, receives land only in ghost rows, and the
    ghost rows cover the widest fused-pass cone (14 rows on level 0 for the
    cross-cycle pass, 7 on the others) wherever a neighbour exists;
  * the all-gather rows of the first replicated level tile [0, n_la) in rank
    order and are exactly the coarse rows each rank's restriction writes.
"""
import pytest

from hpcclassmultigridproject_amd import _lib
from hpcclassmultigridproject_amd import dist as mgd

CONE = {0: 14}      # level 0: the cross-cycle pass (kernels.hip XCfg: 2K + 2K+1 + 1)
CONE_OTHER = 7      # a K=3 fused pass + residual: E = 2K + 1


@pytest.mark.parametrize("N,L", [(1024, 6), (4096, 3), (16384, 9), (65536, 11)])
@pytest.mark.parametrize("G", [2, 4, 8, 16])
def test_exchange_plan_pairs_and_covers_cones(N, L, G):
    parts = {r: [mgd.partition(N, L, G, r, l) for l in range(L)] for r in range(G)}
    la = parts[0][0][2]
    for l in range(la):
        n = N >> l
        plans = {r: mgd.exchange_plan(N, L, G, r, l) for r in range(G)}
        for r in range(G):
            ra, rb, _ = parts[r][l]
            peers = sorted(x[0] for x in plans[r])
            assert peers == [p for p in (r - 1, r + 1) if 0 <= p < G]
            for peer, s0, sn, r0, rn in plans[r]:
                assert sn > 0 and rn > 0
                assert ra <= s0 and s0 + sn <= rb, "send outside owned rows"
                assert r0 + rn <= ra or r0 >= rb, "receive into owned rows"
                assert 0 <= r0 and r0 + rn <= n + 1
                back = [x for x in plans[peer] if x[0] == r]
                assert len(back) == 1
                _, ps0, psn, pr0, prn = back[0]
                assert (pr0, prn) == (s0, sn), "peer receives other rows than sent"
                assert (ps0, psn) == (r0, rn), "peer sends other rows than received"
                # the ghost band is adjacent to the owned rows and covers the cone
                cone = CONE.get(l, CONE_OTHER)
                if peer < r:
                    assert r0 + rn == ra and rn >= min(cone, ra)
                else:
                    assert r0 == rb and rn >= min(cone, n + 1 - rb)


@pytest.mark.parametrize("N,L", [(1024, 6), (16384, 9), (65536, 11)])
@pytest.mark.parametrize("G", [2, 4, 8])
def test_gather_plan_tiles_the_replicated_level(N, L, G):
    got = [mgd.gather_plan(N, L, G, r) for r in range(G)]
    la = got[0][0]
    assert all(g[0] == la for g in got)
    if la == 0:   # nothing partitioned (blocks would be < dist_min_rows): no gather
        return
    nl = N >> la
    rows = [(r0, q) for _, r0, q in got]
    assert rows[0][0] == 0 and all(q == rows[0][1] for _, q in rows)
    for (a0, q0), (a1, _) in zip(rows, rows[1:]):
        assert a1 == a0 + q0
    assert rows[-1][0] + rows[-1][1] == nl   # row nl is the boundary (never read)
    # each rank contributes exactly the coarse rows I = r/2, r even, r in its
    # level la-1 block [ra, rb) (the fused restriction's writes)
    for r, (r0, q) in enumerate(rows):
        ra, rb, _ = mgd.partition(N, L, G, r, la - 1)
        own = sorted({i // 2 for i in range(ra, rb) if i % 2 == 0 and i // 2 < nl})
        assert own == list(range(r0, r0 + q))


def test_plan_rejects_bad_arguments():
    with pytest.raises(_lib.MGXError):
        mgd.exchange_plan(1000, 5, 2, 0, 0)   # n not a power of two
    with pytest.raises(_lib.MGXError):
        mgd.exchange_plan(1024, 5, 3, 0, 0)   # world not a power of two
    assert mgd.exchange_plan(1024, 6, 1, 0, 0) == []
