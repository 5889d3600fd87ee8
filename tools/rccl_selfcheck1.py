import sys, os
sys.path.insert(0, '.')
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29555")
os.environ.setdefault("RANK", "0"); os.environ.setdefault("WORLD_SIZE", "1")
import torch.distributed as dist
from hpcclassmultigridproject_amd import dist as mgdist
dist.init_process_group("gloo")
print(mgdist.rccl_selfcheck(1, 0, 0), flush=True)
dist.destroy_process_group()
