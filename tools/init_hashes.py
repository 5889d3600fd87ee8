import sys, hashlib; sys.path.insert(0,'.')
import hpcclassmultigridproject_amd as pkg
from oracle import oracle as O
for N in (128, 1024, 4096):
    a = pkg.init_problem(N)
    b = O.init_problem(N)
    print(N, [hashlib.sha256(x.tobytes()).hexdigest()[:12] for x in a], [hashlib.sha256(x.tobytes()).hexdigest()[:12] for x in b], flush=True)
