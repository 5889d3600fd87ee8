# A/B of smoother variants in one process (bench-like loop)
import sys, time, json
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
N, L = 16384, 9
dt = 1.0/N/10
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
res = {}
for rnd in range(2):
    for sm, fu in [(0,3),(0,2),(0,1),(2,3)]:
        mg = pkg.Multigrid(N, L, dt, -4e-4, smoother=sm, fuse=fu, device=0)
        mg.upload(u0, v1, v2); mg.rhs(); mg.run_cycles(1); mg.synchronize()
        mg.profile(True)
        t = time.perf_counter(); r = mg.run_cycles(5); mg.synchronize(); el = (time.perf_counter()-t)/5
        d = {"ms": round(el*1e3, 3), "res": r}
        for k, name in _lib.KERNEL_NAMES.items():
            n, ms, b = mg.profile_get(k, 0)
            if n: d[name+"_L0_ms"] = round(ms/n, 4); d[name+"_L0_algGBs"] = round(b/n/(ms/n*1e-3)/1e9)
            n, ms, b = mg.profile_get(k, -1)
            if n: d[name+"_all_ms_step"] = round(ms/5, 3)
        mg.close()
        res[f"{sm},{fu},r{rnd}"] = d
        print(f"{sm},{fu},r{rnd}", json.dumps(d), flush=True)
