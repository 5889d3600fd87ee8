"""libmgx's RCCL transport with real peers (2 processes, 2 GPUs).

tests/test_gpu_dist.py covers the partitioned solver on virtual ranks (the
same partition and exchange plan, exchanges as device copies) and RCCL on a
size-1 communicator; RCCL refuses two ranks on one GPU.  This test needs two
visible GPUs: it launches tests/rccl_worker.py under torch.distributed.run
with --nproc-per-node 2, whose ranks run the partitioned V-cycle over RCCL
(ghost send/recv, all-gather into the replicated levels, norm all-reduce,
download all-gather + broadcast), with and without the overlapped exchange,
and compare with a one-GPU context: u bitwise, norms to 1e-11.  bench.py
runs the same check before timing whenever it runs on N > 1 GPUs
("rccl_parity" in its JSON line).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpus():
    import torch
    return torch.cuda.device_count()   # counting does not initialise the GPU


@pytest.mark.skipif(_gpus() < 2, reason="needs 2 visible GPUs (RCCL refuses 2 ranks on 1 GPU)")
def test_rccl_two_ranks_bitwise_vs_one_gpu(tmp_path):
    out = tmp_path / "verdict.json"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29517",
           os.path.join(ROOT, "tests", "rccl_worker.py"), str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(out.read_text())
    assert res["partitioned_levels"] >= 2, res
    assert res["bitwise"] and res["passed"], res
