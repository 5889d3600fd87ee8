"""Cost of the row partition on one GPU: ms per V-cycle (+norm) for the single
context vs G virtual ranks (mgx_create_local_dist), per-kind device times.
The virtual ranks run one after another on one stream, so G parts ~ 1 GPU's
work + the partition overheads (ghost rows recomputed, exchanges, more
launches, replicated coarse levels G times).
    python tools/ab_dist.py [--N 16384 --L 9] [--parts 1,2,4,8] [--cycles 5] [--tower correct]
                            [--knob key=v1,v2]   (a process-wide tuning key to compare)
                            [--fp fma|bitwise]   (mgx_options.fp_mode, default fma)"""
import argparse, json, sys, time
sys.path.insert(0, '.')
import hpcclassmultigridproject_amd as pkg
from hpcclassmultigridproject_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument('--N', type=int, default=16384)
ap.add_argument('--L', type=int, default=9)
ap.add_argument('--parts', default='1,2,4,8')
ap.add_argument('--cycles', type=int, default=5)
ap.add_argument('--rounds', type=int, default=2)
ap.add_argument('--min-rows', default='256')
ap.add_argument('--overlap', default='0', help='dist_overlap values to compare, e.g. 0,1')
ap.add_argument('--knob', default=None, help='key=v1,v2: a tuning key to compare')
ap.add_argument('--fp', choices=['bitwise', 'fma'], default='fma')
ap.add_argument('--tower', choices=['reference', 'correct'], default='reference',
                help='correct: no whole-grid staging buffers (N=65536 on one GPU)')
a = ap.parse_args()
N, L = a.N, a.L
dt = 1.0 / N / 10
u0, v1, v2 = pkg.init_problem(N, nthreads=16)
kkey, kvals = (a.knob.split('=')[0], [int(x) for x in a.knob.split('=')[1].split(',')]) \
    if a.knob else (None, [None])
for rnd in range(a.rounds):
 for kv in kvals:
  if kkey:
      _lib.set_tuning(kkey, kv)
  for mr in (int(x) for x in a.min_rows.split(',')):
   _lib.set_tuning("dist_min_rows", mr)
   for ov in (int(x) for x in a.overlap.split(',')):
    _lib.set_tuning("dist_overlap", ov)
    for G in [int(x) for x in a.parts.split(',')]:
        if G == 1 and ov:
            continue
        mg = pkg.Multigrid(N, L, dt, -4e-4, device=0, local_parts=G if G > 1 else 0,
                           fp_mode=_lib.FP_FMA if a.fp == 'fma' else _lib.FP_BITWISE,
                           tower_mode=_lib.TOWER_CORRECT if a.tower == 'correct'
                           else _lib.TOWER_REFERENCE)
        if G > 1 and a.tower == 'correct':   # row-block upload (no whole-grid staging)
            mg.upload_rows([pkg.init_problem_rows(N, lo, hi + 1, nthreads=16)
                            for lo, hi in (mg.dist_rows(p) for p in range(G))])
        else:
            mg.upload(u0, v1, v2)
        mg.rhs(); mg.run_cycles(1); mg.synchronize()
        mg.profile_reset(); mg.profile(True)
        t = time.perf_counter(); r = mg.run_cycles(a.cycles); mg.synchronize()
        ms = (time.perf_counter() - t) / a.cycles * 1e3
        d = {"knob": f"{kkey}={kv}" if kkey else None, "min_rows": mr, "overlap": ov, "G": G,
             "ms": round(ms, 3),
             "ms_per_rank": round(ms / G, 3), "la": mg.dist_info()[2], "res": r}
        for kind, name in _lib.KERNEL_NAMES.items():
            n, kms, _ = mg.profile_get(kind, -1)
            if n: d[name] = round(kms / a.cycles, 4)
        lv = []
        for l in range(L):
            t = 0.0
            for kind in _lib.KERNEL_NAMES:
                n, kms, _ = mg.profile_get(kind, l)
                t += kms
            lv.append(round(t / a.cycles, 4))
        d["per_level_ms"] = lv
        mg.profile(False); mg.close()
        print(rnd, json.dumps(d), flush=True)
