"""Step through the world-size-1 RCCL partitioned context (debug helper)."""
import faulthandler
import sys

import numpy as np

sys.path.insert(0, ".")
faulthandler.enable()
from hpcclassmultigridproject_amd import Multigrid, dist, init_problem  # noqa: E402

N, L = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 4
uid = dist.unique_id()
print("uid ok", flush=True)
u0, v1, v2 = init_problem(N)
mg = Multigrid(N, L, 1.0 / N / 10, -4e-4, world=1, rank=0, unique_id=uid)
print("created", mg.dist_info(), flush=True)
mg.upload(u0, v1, v2)
print("uploaded", flush=True)
mg.rhs()
print("rhs", flush=True)
print("cycle", mg.run_cycles(1), flush=True)
print("resnorm", mg.residual_norm(0), flush=True)
u = mg.download()
print("downloaded", np.abs(u).sum(), flush=True)
mg.close()
print("closed", flush=True)
