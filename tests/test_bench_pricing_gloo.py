"""CPU, 2 ranks over gloo: bench.price_partitions -- the N > 1 warm-up's
loop over the (dist_min_rows, dist_overlap) candidates -- with a stand-in
context whose cycle cost depends on the rank and the knobs.  Every rank must
time the same candidates in the same order (their collectives pair up), take
the max over ranks, rebuild a context only when the rows change, and end with
the winner's context."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_WORKER = r"""
import json, os, sys, time
sys.path.insert(0, {root!r})
import torch, torch.distributed as dist
import bench
dist.init_process_group("gloo")
rank = dist.get_rank()
state = {{"overlap": None}}
log = []
# per-cycle seconds: rank 1 is slow on overlap 2, so the max over ranks must
# rule that pair out although rank 0 alone would pick it
COST = {{(128, 0): 0.004, (128, 1): 0.003, (128, 2): 0.001, (256, 0): 0.005, (256, 1): 0.004,
        (256, 2): 0.001, (512, 0): 0.006, (512, 1): 0.005, (512, 2): 0.001}}

class Ctx:
    def __init__(self, rows):
        self.rows, self.closed = rows, False
        log.append(("create", rows))
    def run_cycles(self, k):
        assert not self.closed
        c = COST[(self.rows, state["overlap"])]
        if rank == 1 and state["overlap"] == 2:
            c = 0.02
        time.sleep(c * k)
    def synchronize(self):
        pass
    def close(self):
        self.closed = True
        log.append(("close", self.rows))

def barrier():
    dist.barrier()

def max_over_ranks(x):
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

def set_overlap(ov):
    state["overlap"] = ov
    log.append(("overlap", ov))

cands = bench.pricing_candidates("auto", "auto", 16384, None)
mg = Ctx(cands[-1][0])
mg, cur, br, bo, ab = bench.price_partitions(mg, cands[-1][0], cands, lambda r, w: Ctx(r),
                                             barrier, max_over_ranks, set_overlap)
out = {{"rank": rank, "best": [br, bo], "cur": cur, "ctx_rows": mg.rows, "closed": mg.closed,
       "ab": ab, "log": log}}
with open({out!r} + f".{{rank}}", "w") as f:
    json.dump(out, f)
dist.destroy_process_group()
"""


def test_price_partitions_two_ranks(tmp_path):
    out = str(tmp_path / "res")
    script = tmp_path / "worker.py"
    script.write_text(_WORKER.format(root=ROOT, out=out))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29641", WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(2)]
    for p in procs:
        _, err = p.communicate(timeout=120)
        assert p.returncode == 0, err[-3000:]
    res = [json.load(open(f"{out}.{r}")) for r in range(2)]
    for r in res:
        # (128, 2) is fastest on rank 0 alone; the max over ranks picks (128, 1)
        assert r["best"] == [128, 1] and r["cur"] == 128 and r["ctx_rows"] == 128
        assert not r["closed"]
        assert set(r["ab"]) == {f"{a}:{b}" for a in (128, 256, 512) for b in (0, 1, 2)}
        # rows descending: the first (512) context is the one passed in; one
        # rebuild per other rows value, the last (128) kept (no extra build)
        creates = [x for x in r["log"] if x[0] == "create"]
        assert creates == [["create", 512], ["create", 256], ["create", 128]], creates
    assert res[0]["ab"] == res[1]["ab"]   # max over ranks: identical on every rank
    assert res[0]["log"] == res[1]["log"]
