"""Time steps at N=16384: mgx_step (compute_rhs fused with mg_outer's initial
norm) vs rhs() + mg_outer() (two passes), interleaved.
    python tools/step_time.py [--N 16384 --L 9 --steps 3 --rounds 2]"""
import argparse, sys, time
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
ap = argparse.ArgumentParser()
ap.add_argument('--N', type=int, default=16384)
ap.add_argument('--L', type=int, default=9)
ap.add_argument('--steps', type=int, default=3)
ap.add_argument('--rounds', type=int, default=2)
a = ap.parse_args()
N, L = a.N, a.L
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
mg = pkg.Multigrid(N, L, 1.0 / N / 10, -4e-4, device=0)
for rnd in range(a.rounds):
    for fused in (False, True):
        mg.upload(u0, v1, v2)
        mg.synchronize()
        t = time.perf_counter()
        cyc = []
        for _ in range(a.steps):
            if fused:
                cyc.append(mg.step(1e-6))
            else:
                mg.rhs()
                cyc.append(mg.mg_outer(1e-6)[0])
        mg.synchronize()
        ms = (time.perf_counter() - t) / a.steps * 1e3
        print(rnd, "fused" if fused else "separate", f"{ms:.3f} ms/step", "cycles", cyc, flush=True)
