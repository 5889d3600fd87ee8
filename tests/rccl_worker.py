"""Worker of tests/test_gpu_rccl.py: one rank of a torch.distributed.run job.

Runs libmgx's RCCL transport with real peers (hpcclassmultigridproject_amd.
dist.rccl_selfcheck: partitioned V-cycles with and without the overlapped
exchange, vs a one-GPU context on rank 0) and writes rank 0's verdict as JSON
to the path in argv[1]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch.distributed as dist  # noqa: E402

from hpcclassmultigridproject_amd import dist as mgdist  # noqa: E402

rank, world, local = mgdist.env_rank()
dist.init_process_group("gloo")
res = mgdist.rccl_selfcheck(world, rank, local)
if rank == 0:
    with open(sys.argv[1], "w") as f:
        json.dump(res, f)
dist.barrier()
dist.destroy_process_group()
