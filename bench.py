#!/usr/bin/env python3
"""Headline benchmark: V-cycle grid-point-updates/sec at N=16384 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A step = one V-cycle (mg_inner, multigrid.cpp:17-92) + the residual and norm
mg_outer computes after it (multigrid.cpp:112-113), with a fixed cycle count
(no tolerance stop).  Workload: the reference problem (Gaussian u0,
rotating velocity, nu=-4e-4, dt=dx/10) at N=16384, L=9 levels (coarsest 64),
3 pre/post RB-GS sweeps, fp64; inputs resident in HBM before the timed region.

value = (N-1)^2 * steps / max-over-ranks seconds (whole job).
Multi-GPU (torch.distributed.run, one rank per GPU): the north star's strong
scaling -- the same N=16384 grid row-partitioned over the ranks (libmgx RCCL
halo exchange, replicated coarse levels), "scaling":
"strong".  --weak instead doubles N (and adds a level) per 4x ranks, so the
points per GPU stay within 2x of the 1-GPU run, "scaling": "weak"
(configs[4], N=65536 on 8 GPUs: --N 65536 --levels 11; above N=16384 each
rank initialises and uploads only its own rows, with the correct velocity
tower, so no host or GPU ever holds the whole grid).
roofline: the dominant kernel (largest device time: the finest level's fused
cross-cycle pass) with achieved = its COMPULSORY bytes per launch (every array
the pass must read or write, once: u, rhs, v1, v2 and the coarse u read, u_pre
(+ u_post on the cycle whose solution is kept) and the coarse rhs written;
DESIGN.md section 5) / its mean duration (HIP events on the context stream,
inside the timed region); frac = achieved / 8 TB/s.  The SURVEY 8d per-op
canonical bytes the same launch replaces (12 reference ops per HBM pass) are
reported beside it as canonical_equiv_GBs, never as the fraction.
traffic = its measured HBM bytes per launch (rocprofv3 PMC, the
profiles/*_hbm_traffic.json whose kernels.hip hash matches the built source;
null with a reason when none does).
cpu_baseline: rank 0, N=1 only: the reference's own mg_inner (oracle/_ref,
built from the unmodified sources), OpenMP tasks: the reference Makefile's
-O0 build and an -O3 build, each serial and on all host cores this process may
use (sched affinity, capped by the cgroup CPU quota); value = the fastest.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s HBM3E
# (kind, level) -> kernel (template instance) of the default config, for the
# PMC traffic summary committed under profiles/ (tools/profile_round.sh)
# (the cross pass is two launches: the unguarded interior kernel and the
# guarded edge kernel; their traffic is summed)
KERNEL_IDS = {(8, 0): ("mgx::k_xsmooth<4, 3, false, false, true, false>",
                       "mgx::k_xsmooth<1, 3, true, false, true, false>"),
              (0, 0): ("mgx::k_wsmooth<4, 3, 4, true>",),
              (7, 0): ("mgx::k_wsmooth<4, 3, 10, true>",)}
KERNELS_HIP = os.path.join(ROOT, "hpcclassmultigridproject_amd", "csrc", "kernels.hip")


def kernels_sha():
    import hashlib
    return hashlib.sha256(open(KERNELS_HIP, "rb").read()).hexdigest()


def traffic_profile():
    """(path, kernels) of the newest profiles/*_hbm_traffic.json collected from
    the kernels.hip that is built now, or (None, reason)."""
    import glob
    sha = kernels_sha()
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm_traffic.json")),
                   key=os.path.getmtime, reverse=True)
    for f in files:
        d = json.load(open(f))
        if d.get("kernels_hip_sha256") == sha:
            return os.path.relpath(f, ROOT), d["kernels"]
    return None, (f"no profiles/*_hbm_traffic.json matches kernels.hip sha256 {sha[:12]} "
                  "(regenerate with tools/profile_round.sh)")


def lookup_traffic(knames, field="hbm_bytes"):
    """HBM bytes (or another per-dispatch PMC field) of the finest-level
    instances (largest traffic) of the kernels in knames, summed (one launch of
    the op = one dispatch of each)."""
    path, kernels = traffic_profile()
    if path is None:
        return None, None, kernels
    keys, total = [], 0.0
    for kname in knames:
        best = None
        for key, v in kernels.items():
            if key.split(" grid=")[0] == kname and (best is None or v["hbm_bytes"] > best[1]):
                best = (key, v["hbm_bytes"], v.get(field))
        if best is None or best[2] is None:
            return None, None, f"{kname} ({field}) not in {path}"
        keys.append(best[0])
        total += best[2]
    return " + ".join(keys), total, path


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--levels", type=int, default=9)
    ap.add_argument("--nsmooth", type=int, default=3)
    ap.add_argument("--smoother", type=int, default=0,
                    help="0 temporally blocked passes, 1 two-colour, 2 one-pass single sweeps")
    ap.add_argument("--fuse", type=int, default=3, help="smoother 0: sweeps per HBM pass")
    ap.add_argument("--cpu-baseline", choices=["auto", "off", "reference", "port"],
                    default="auto")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the all-cores CPU legs (0: every host CPU this "
                         "process may use)")
    ap.add_argument("--weak", action="store_true",
                    help="multi-GPU: grow N with the GPU count (N*2 per 4x GPUs) instead of "
                         "partitioning the same grid")
    ap.add_argument("--row-upload", choices=["auto", "on", "off"], default="auto",
                    help="multi-GPU: each rank builds only its rows (auto: N > 16384)")
    ap.add_argument("--overlap", choices=["auto", "0", "1", "2"], default="auto",
                    help="N > 1: dist_overlap for the timed region; auto = price 0 / 1 / 2 "
                         "in the warm-up (3 cycles each, max over ranks) and keep the fastest")
    ap.add_argument("--rccl-check", type=int, default=1,
                    help="N > 1: first check libmgx's RCCL path bitwise vs one GPU (N=4096)")
    ap.add_argument("--no-generic", action="store_true",
                    help="skip the comparison run with the generic (2-D) velocity path")
    ap.add_argument("--no-profile", action="store_true",
                    help="do not record per-kernel HIP events in the timed region")
    ap.add_argument("--sweep", nargs=2, type=int, metavar=("NMIN", "NMAX"),
                    help="instead of the bench line: the 100-step time stepper for N = NMIN.."
                         "NMAX (powers of two) on the GPU and the reference on the host, "
                         "serial and all usable cores; writes cudatime.txt, serialtime.txt, "
                         "omptime.txt ('N<TAB>seconds', what speedupplot.py reads)")
    ap.add_argument("--sweep-out", default="", help="--sweep: output file prefix")
    return ap.parse_args()


def host_cpus():
    """CPUs this process may use (affinity, capped by the cgroup v2 quota) and
    what the host reports."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return {"usable": usable, "affinity": aff, "nproc_host": os.cpu_count(),
            "cgroup_quota_cpus": quota, "model": model,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(args):
    """The reference's own mg_inner on the host: -O0 (reference Makefile) and
    -O3 builds, serial and all usable cores.  Bounded sample: one V-cycle each;
    the serial legs at N/2 (a quarter of the work, same per-unknown loops) so
    the whole baseline stays ~30 s."""
    from oracle import oracle as O
    cpus = host_cpus()
    allc = args.cpu_threads or cpus["usable"]
    N, L, nu = args.N, args.levels, -4e-4
    kind = args.cpu_baseline
    if kind == "auto":
        kind = "reference" if O.ref_available() else "port"
    runs = []
    if kind == "reference":
        legs = [("O3", allc, N, L), ("O0", allc, N, L), ("O3", 1, N // 2, L - 1),
                ("O0", 1, N // 2, L - 1)]
        for opt, th, n, lv in legs:
            if opt == "O3" and not O.ref_o3_available():
                continue
            secs, setup, res = O.ref_time_vcycles(n, lv, nu, 1, th, opt=opt)
            runs.append({"build": opt, "threads": th, "N": n, "levels": lv,
                         "seconds_per_vcycle": round(secs, 4),
                         "value": (n - 1) ** 2 / secs})
        flags = {"O0": "-O0 -fopenmp (reference Makefile flags)",
                 "O3": "-O3 -march=x86-64-v3 -fopenmp"}
    else:
        O.set_threads(allc)
        u0, v1, v2 = O.init_problem(N)
        dt = 1.0 / N / 10
        t = O.Tower(u0, v1, v2, N, L)
        del u0, v1, v2
        O.compute_rhs(t.ufine, N, t.level("v1", 0), t.level("v2", 0), dt, nu, 1.0 / N,
                      rhs=t.rhsfine)
        t0 = time.perf_counter()
        t.mg_inner(dt, nu)
        O.residual(t.ufine, t.rhsfine, N, t.level("v1", 0), t.level("v2", 0), dt, nu, 1.0 / N,
                   res=t.tmp)
        secs = time.perf_counter() - t0
        runs.append({"build": "port -O2", "threads": allc, "N": N, "levels": L,
                     "seconds_per_vcycle": round(secs, 4), "value": (N - 1) ** 2 / secs})
        flags = {"port -O2": "oracle/mg_oracle.c restatement, gcc -O2 -fopenmp"}
    best = max((r for r in runs if r["N"] == N), key=lambda r: r["value"])
    return {"value": best["value"], "unit": "grid-point-updates/s", "cores": best["threads"],
            "kind": kind, "build": flags[best["build"]],
            "seconds_per_vcycle": best["seconds_per_vcycle"], "runs": runs, "host": cpus,
            "sample": f"1 V-cycle (mg_inner + residual + norm) per leg, OpenMP tasks of the "
                      f"reference; all-core legs at N={N}, L={L}, nu_smooth=3 on "
                      f"{allc} threads; serial legs at N={N // 2}, L={L - 1} (per-unknown "
                      f"rate); value = the fastest leg at N={N}"}


def sweep(args):
    """speedupplot.py's three inputs (/root/reference/speedupplot.py:10,25,40):
    wall seconds of the 100-step time stepper per N, GPU (mgx_timestepper, as
    mg_timer.cu times it: setup + steps + copy back) and the reference
    timestepper on the host (oracle/_ref, the cpu_baseline leg's build), 1
    thread and every usable core (multigrid.cpp:244-258 method)."""
    import hpcclassmultigridproject_amd as pkg
    from oracle import oracle as O
    if not O.ref_available():
        sys.exit("--sweep needs the compiled reference (oracle/_ref)")
    cores = host_cpus()["usable"]
    files = {k: open(args.sweep_out + k + "time.txt", "w") for k in ("cuda", "serial", "omp")}
    out = {"sweep": [], "cores": cores}
    N = args.sweep[0]
    while N <= args.sweep[1]:
        L = max(1, int(math.log2(N)) - 4)
        dx = 1.0 / N
        dt, nu = dx / 10, -4e-4
        T = 100 * dt
        u0, v1, v2 = pkg.init_problem(N)
        uT = np.empty_like(u0)
        t0 = time.perf_counter()
        pkg.timestepper(uT, u0, v1, v2, nu, L, N, dt, T, dx, 1e-6)
        tg = time.perf_counter() - t0
        row = {"N": N, "cuda": tg}
        for key, th in (("serial", 1), ("omp", cores)):
            t0 = time.perf_counter()
            ref = O.ref_timestepper(u0, v1, v2, nu, L, N, dt, T, dx, nthreads=th)
            row[key] = time.perf_counter() - t0
            row[key + "_bitwise"] = bool(np.array_equal(ref, uT))
        for k, f in files.items():
            f.write(f"{N}\t{row[k]:f}\n")
            f.flush()
        out["sweep"].append(row)
        N *= 2
    for f in files.values():
        f.close()
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    if args.sweep:
        return sweep(args)
    import torch
    import torch.distributed as dist

    import hpcclassmultigridproject_amd as pkg
    from hpcclassmultigridproject_amd import _lib

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("for --gpus > 1 launch with torch.distributed.run --nproc-per-node N")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if world > 1:
            dist.barrier()

    rccl_check = None
    if world > 1 and args.rccl_check:
        # libmgx's own RCCL transport with real peers vs a one-GPU context,
        # bitwise (small problem, before and outside the timed region)
        from hpcclassmultigridproject_amd import dist as mgdist
        rccl_check = mgdist.rccl_selfcheck(world, rank, local)

    N, L = args.N, args.levels
    if args.weak and world > 1:
        # points per GPU ~ constant: N grows by 2 per 4x ranks (power of two)
        g = 1
        while 4 * g <= world:
            N, L, g = 2 * N, L + 1, 4 * g
    nu = -4e-4
    dt = 1.0 / N / 10
    dist_kw = {}
    if world > 1:
        from hpcclassmultigridproject_amd import dist as mgdist
        dist_kw = dict(world=world, rank=rank, unique_id=mgdist.broadcast_unique_id())
    # row-block upload: each rank initialises and uploads only its rows (the
    # whole grid never exists on one host/GPU: C5, N=65536 on 8 GPUs); it needs
    # the correct velocity tower (the reference tower reads the whole grid)
    row_upload = world > 1 and (args.row_upload == "on" or
                                (args.row_upload == "auto" and N > 16384))
    # (and above N=16384 everywhere: the reference tower's two whole-grid
    # staging buffers, 2 x 34 GB at N=65536, do not fit beside the towers on
    # one GPU; the reference's own int indexing overflows there)
    tower = (pkg._lib.TOWER_CORRECT if row_upload or N > 16384
             else pkg._lib.TOWER_REFERENCE)
    mg = pkg.Multigrid(N, L, dt, nu, nsmooth=args.nsmooth, device=local,
                       smoother=args.smoother, fuse=args.fuse, tower_mode=tower, **dist_kw)
    la = mg.dist_info()[2]
    if row_upload:
        lo, hi = mg.dist_rows(0)
        mg.upload_rows([pkg.init_problem_rows(N, lo, hi + 1, nthreads=16)])
    else:
        u0, v1, v2 = pkg.init_problem(N, nthreads=16)
        mg.upload(u0, v1, v2)
        del u0, v1, v2
    mg.rhs()
    for _ in range(args.warmup):
        mg.run_cycles(1)
    mg.synchronize()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    overlap_ab = None
    if world > 1:
        # price the exchange schedules on this machine (untimed warm-up): the
        # early level-0 exchange behind the coarse levels pays over xGMI but not
        # on one GPU's virtual ranks
        if args.overlap == "auto":
            overlap_ab = {}
            for ov in (0, 1, 2):
                _lib.set_tuning("dist_overlap", ov)
                mg.run_cycles(1)
                mg.synchronize()
                barrier()
                t0 = time.perf_counter()
                mg.run_cycles(3)
                mg.synchronize()
                overlap_ab[ov] = round(max_over_ranks(time.perf_counter() - t0) / 3 * 1e3, 4)
            best_ov = min(overlap_ab, key=overlap_ab.get)
        else:
            best_ov = int(args.overlap)
        _lib.set_tuning("dist_overlap", best_ov)
        mg.run_cycles(1)
        mg.synchronize()
    mg.profile_reset()
    if not args.no_profile:
        # HIP events around the finest-level launches only (the dominant
        # kernels); events around every small-level launch would cost ~7%
        mg.profile(True, finest_only=True)

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # K steps = K V-cycles, each followed by its residual norm (read back per
    # cycle, as mg_outer does); the solution after the K-th is materialised
    res = mg.run_cycles(args.steps)
    mg.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0)

    # dominant kernel = the finest-level (kind) with the largest device time
    # in the timed region
    best = None
    for kind in _lib.KERNEL_NAMES:
        n, ms, b, cb = mg.profile_get_ex(kind, 0)
        if n and (best is None or ms > best[3]):
            best = (kind, 0, n, ms, b, cb)
    mg.profile(False)

    # per-kernel, per-level breakdown: a few more cycles, every launch timed
    # (after the timed region, so its event overhead is not in `value`)
    kernels = {}
    if not args.no_profile:
        prof_steps = 3
        mg.profile_reset()
        mg.profile(True)
        mg.run_cycles(prof_steps)
        for kind, name in _lib.KERNEL_NAMES.items():
            n, ms, b, cb = mg.profile_get_ex(kind, -1)
            if n:
                kernels[name] = {"launches_per_step": n / prof_steps,
                                 "ms_per_step": round(ms / prof_steps, 4),
                                 "compulsory_GBs": round(cb / (ms * 1e-3) / 1e9, 1)
                                 if ms > 0 else None,
                                 "canonical_equiv_GBs": round(b / (ms * 1e-3) / 1e9, 1)
                                 if ms > 0 else None}
                for lvl in range(L):
                    nl, msl, bl = mg.profile_get(kind, lvl)
                    if nl:
                        kernels[name][f"L{lvl}_ms_per_step"] = round(msl / prof_steps, 4)
        mg.profile(False)
    import ctypes
    fac = ctypes.c_int(0)
    if world == 1:
        _lib.check(_lib.lib().mgx_velocity_factored(mg.handle, ctypes.byref(fac)))
    mg.close()

    # the same V-cycle with the generic velocity path (2-D v1 / v2 on every
    # row of every level: sep_velocity = zero_rows = 0), for comparison: the
    # headline reads the reference flow's exact rank-1 factors on level 0 and
    # skips the coarse levels' all-zero velocity rows
    generic = None
    if world == 1 and not args.no_generic:
        keys = {k: _lib.get_tuning(k) for k in ("sep_velocity", "zero_rows")}
        try:
            for k in keys:
                _lib.set_tuning(k, 0)
            g = pkg.Multigrid(N, L, dt, nu, nsmooth=args.nsmooth, device=local,
                              smoother=args.smoother, fuse=args.fuse, tower_mode=tower)
            u0, v1, v2 = pkg.init_problem(N, nthreads=16)
            g.upload(u0, v1, v2)
            del u0, v1, v2
            g.rhs()
            g.run_cycles(2)
            g.synchronize()
            t0 = time.perf_counter()
            g.run_cycles(args.steps)
            g.synchronize()
            gms = (time.perf_counter() - t0) / args.steps * 1e3
            g.close()
            generic = {"ms_per_step": round(gms, 4),
                       "value": (N - 1) ** 2 / (gms * 1e-3),
                       "note": "sep_velocity=0, zero_rows=0: every velocity row read from HBM"}
        finally:
            for k, v in keys.items():
                _lib.set_tuning(k, v)

    roof = None
    if best:
        kind, lvl, n0, ms0, b0, cb0 = best
        # achieved = compulsory bytes per launch (each array the fused pass must
        # read or write, once) / live mean duration; the per-op canonical bytes
        #  of the reference ops it replaces go in canonical_equiv_GBs
        per_launch = cb0 / n0
        avg_s = ms0 * 1e-3 / n0
        achieved = per_launch / avg_s / 1e9
        # the committed PMC traffic is per launch of the single-GPU pass; a
        # rank's row block moves a fraction of it, so it is not reused there
        ids = KERNEL_IDS.get((kind, lvl)) if (N, L, args.nsmooth, args.smoother, args.fuse,
                                              world) == (16384, 9, 3, 0, 3, 1) else None
        kname, traffic, tsrc = (None, None, "no committed PMC profile for this configuration")
        if ids:
            kname, traffic, tsrc = lookup_traffic(ids)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": f"{_lib.KERNEL_NAMES[kind]} level {lvl}"
                          + (f" = {kname}" if kname else ""),
                "compulsory_bytes_per_launch": per_launch,
                "avg_launch_ms": round(avg_s * 1e3, 4),
                "canonical_bytes_per_launch": b0 / n0,
                "canonical_equiv_GBs": round(b0 / n0 / avg_s / 1e9, 1)}
        if traffic:
            # measured HBM bytes (rocprofv3 PMC, profiles/) / live mean duration
            roof["traffic_source"] = tsrc
            roof["hbm_GBs"] = round(traffic / avg_s / 1e9, 1)
            roof["hbm_frac"] = round(traffic / avg_s / 1e9 / HBM_PEAK_GBS, 4)
            roof["traffic_over_compulsory"] = round(traffic / per_launch, 3)
            # the pass is bound by its instruction stream more than by bytes:
            # VALU instructions per launch (PMC SQ_INSTS_VALU, same profile)
            # against the issue capacity in its live duration (one wave
            # instruction per 4 cycles per SIMD, 1024 SIMDs, 2.4 GHz peak clock:
            # a lower bound on the busy fraction)
            _, valu, _ = lookup_traffic(ids, "SQ_INSTS_VALU")
            if valu:
                cap = 1024 * avg_s * 2.4e9 / 4
                roof["valu"] = {"insts_per_launch": valu, "issue_capacity": round(cap),
                                "issue_frac": round(valu / cap, 4),
                                "note": "VALU wave-instructions / (1024 SIMDs x 2.4 GHz / 4 "
                                        "cycles per wave64 op x live mean duration)"}
        else:
            roof["traffic_null_reason"] = tsrc

    value = (N - 1) ** 2 * args.steps / elapsed
    # SURVEY 8d secondary metric: RB-GS point updates per second
    smoother_pts = sum(2 * args.nsmooth * ((N >> l) - 1) ** 2 for l in range(L - 1))
    if roof is not None and rank == 0:
        # measured ceilings (mgx_stream_bandwidth): a copy, and the smoother's
        # 4-in/1-out stream shape; hbm_frac_of_stream = measured traffic rate
        # over the latter
        roof["copy_ceiling_GBs"] = round(_lib.stream_bandwidth(1 << 30, 1, 10), 1)
        roof["stream5_ceiling_GBs"] = round(_lib.stream_bandwidth(1 << 30, 4, 10), 1)
        roof["achieved_frac_of_stream5"] = round(roof["achieved"] / roof["stream5_ceiling_GBs"], 4)
        if "hbm_GBs" in roof:
            roof["hbm_frac_of_stream5"] = round(roof["hbm_GBs"] / roof["stream5_ceiling_GBs"], 4)
    if roof is not None and fac.value and world == 1:
        # the same pass's bytes if v1, v2 were read as 2-D arrays (the
        # reference algorithm's inputs, SURVEY 8(d): GS reads u, rhs, v1, v2):
        # the velocity factors regenerate them bitwise instead of reading them
        vb = 2.0 * 8.0 * (N + 1) * ((N + 1 + 15) // 16 * 16)
        a2 = (roof["compulsory_bytes_per_launch"] + vb) / (roof["avg_launch_ms"] * 1e-3) / 1e9
        roof["algorithmic_2d_velocity"] = {
            "bytes_per_launch": roof["compulsory_bytes_per_launch"] + vb,
            "GBs": round(a2, 1), "frac": round(a2 / HBM_PEAK_GBS, 4),
            "note": "compulsory bytes with v1, v2 counted as read (they are regenerated "
                    "bitwise from their rank-1 factors instead)"}
    out = {
        "metric": f"V-cycle grid-point-updates/sec at N={N}; achieved HBM GB/s vs peak",
        "value": value, "unit": "grid-point-updates/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "smoother_point_updates_per_s": smoother_pts * args.steps / elapsed,
        "scaling": "single" if world == 1 else ("weak" if args.weak else "strong"),
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: the reference problem (Gaussian u0, rotating velocity), "
                "generated on the host with glibc libm",
        "config": {"workload": f"N={N} fp64 V-cycle, L={L} (coarsest {N >> (L - 1)}), "
                               f"nu_smooth={args.nsmooth}, + residual/norm per step",
                   "N": N, "levels": L, "nsmooth": args.nsmooth,
                   "tower": ("correct (row-block upload)" if row_upload else
                             "correct" if tower == pkg._lib.TOWER_CORRECT else "reference"),
                   "parallelism": (f"row-partition x{world} on levels 0..{la - 1}, "
                                   f"levels {la}..{L - 1} replicated" if world > 1
                                   else "single"),
                   "dist_overlap": _lib.get_tuning("dist_overlap") if world > 1 else None,
                   "overlap_ms_per_cycle": overlap_ab,
                   "last_residual": res},
        "roofline": roof,
        "kernels": kernels,
        "velocity": ("level 0: exact rank-1 factors (sep_velocity); coarse levels: all-zero "
                     "rows from one L2-resident row (zero_rows)" if fac.value else
                     "2-D arrays"),
        "generic_velocity_path": generic,
    }
    if rccl_check is not None:
        out["rccl_parity"] = rccl_check
    if rank == 0 and world == 1 and args.cpu_baseline != "off":
        try:
            out["cpu_baseline"] = cpu_baseline(args)
        except Exception as e:   # the baseline is reported, never fatal
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
