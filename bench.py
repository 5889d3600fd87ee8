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
# kernel (template instances) of the dominant pass of the default config per
# fp_mode, for the PMC traffic summary committed under profiles/
# (tools/profile_round.sh): the cross pass is two launches, the unguarded
# interior kernel and the guarded edge kernel; their traffic is summed.
# k_xsmooth<WPB, K, G, RS, SV, FM>
KERNEL_IDS = {("fma", 8): ("mgx::k_xsmooth<4, 3, false, false, true, true>",
                           "mgx::k_xsmooth<1, 3, true, false, true, true>"),
              ("bitwise", 8): ("mgx::k_xsmooth<4, 3, false, false, true, false>",
                               "mgx::k_xsmooth<1, 3, true, false, true, false>"),
              ("fma-generic", 8): ("mgx::k_xsmooth<4, 3, false, false, false, true>",
                                   "mgx::k_xsmooth<1, 3, true, false, false, true>")}
CSRC = os.path.join(ROOT, "hpcclassmultigridproject_amd", "csrc")
KERNEL_SOURCES = ("stencil.h", "kernels.h", "kernels.hip", "wsmooth.hip", "xsmooth.hip")


def kernels_sha():
    """sha256 of the stencil kernel sources (a PMC profile is reused only while
    they are unchanged)."""
    import hashlib
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update(open(os.path.join(CSRC, f), "rb").read())
    return h.hexdigest()


def loaded_kernels_sha():
    """The kernel-sources sha256 the LOADED libmgx.so was built from
    (mgx_build_id, stamped by csrc/Makefile): what a PMC profile must match."""
    from hpcclassmultigridproject_amd import _lib
    return _lib.build_id()["kernel_sources_sha256"]


def traffic_profile(mode):
    """(path, kernels) of the newest profiles/*_hbm_traffic.json collected from
    the kernel sources the loaded library was built from, in fp mode `mode`, or
    (None, reason)."""
    import glob
    sha = loaded_kernels_sha()
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*hbm_traffic*.json")),
                   key=os.path.getmtime, reverse=True)
    for f in files:
        d = json.load(open(f))
        if d.get("kernel_sources_sha256") == sha and d.get("mode") == mode:
            return os.path.relpath(f, ROOT), d["kernels"]
    return None, (f"no profiles/*_hbm_traffic.json ({mode}) matches the loaded library's "
                  f"kernel sources sha256 {sha[:12]} (regenerate with tools/profile_round.sh)")


def lookup_traffic(knames, mode, field="hbm_bytes"):
    """HBM bytes (or another per-dispatch PMC field) of the finest-level
    instances (largest traffic) of the kernels in knames, summed (one launch of
    the op = one dispatch of each)."""
    path, kernels = traffic_profile(mode)
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
    ap.add_argument("--min-rows", default="auto",
                    help="N > 1: dist_min_rows (levels whose row blocks would be shorter are "
                         "replicated); auto = price the candidates 128 / 256 beside the overlap "
                         "modes in the warm-up (N <= 16384; above it the default 256)")
    ap.add_argument("--rccl-check", type=int, default=1,
                    help="N > 1: first check libmgx's RCCL path bitwise vs one GPU (N=4096)")
    ap.add_argument("--fp-mode", choices=["fma", "bitwise"], default="fma",
                    help="arithmetic of the smoothing passes (mgx_options.fp_mode): fma = "
                         "contracted, within 1e-12 of the reference; bitwise = the reference's "
                         "bits")
    ap.add_argument("--reps", type=int, default=5,
                    help="timed repetitions of --steps cycles; value = the median (SURVEY 8d)")
    ap.add_argument("--no-compare", "--no-generic", action="store_true", dest="no_compare",
                    help="skip the comparison runs (other fp_mode, generic velocity path)")
    ap.add_argument("--no-profile", action="store_true",
                    help="do not record per-kernel HIP events in the timed region")
    ap.add_argument("--sweep", nargs=2, type=int, metavar=("NMIN", "NMAX"),
                    help="instead of the bench line: the 100-step time stepper for N = NMIN.."
                         "NMAX (powers of two) on the GPU and the reference on the host, "
                         "serial and all usable cores; writes cudatime.txt, serialtime.txt, "
                         "omptime.txt ('N<TAB>seconds', what speedupplot.py reads)")
    ap.add_argument("--sweep-out", default="", help="--sweep: output file prefix")
    ap.add_argument("--watchdog-s", type=float, default=300.0,
                    help="N > 1: deadline of each phase that waits on peers (RCCL self-check, "
                         "set-up, overlap pricing, timed region); on expiry the rank prints an "
                         "error JSON line and exits 1 instead of hanging")
    return ap.parse_args()


def velocity_note(mask, correct, L):
    """How the run's passes get v1, v2 (mgx_velocity_factored bit mask)."""
    if not mask:
        return "2-D arrays on every level"
    gen = [l for l in range(1, L) if mask >> l & 1]
    s = "level 0: exact rank-1 factors (sep_velocity)"
    if gen:
        s += f"; levels {gen[0]}-{gen[-1]}: regenerated from them in the 3-sweep marches (vgen"
        s += ", strided: the correct tower)" if correct else ", the reference tower's re-read)"
    if not correct:
        s += "; coarse levels: all-zero rows from one L2-resident row (zero_rows)"
    return s + "; LDS-tile levels and the coarsest solve read the arrays"


class GpuState:
    """Clock, power and temperature of the bench GPU, read-only from the
    amdgpu sysfs / hwmon files of the card whose PCI address is torch's device
    (the box exposes every GPU of its host there).  Sampled right after each
    timed repetition (outside the clock): the hwmon sclk / mclk readings are
    short averages, so they show the clocks the repetition ran at.  Every
    field is optional: a file that cannot be read is left out."""

    def __init__(self, device):
        self.hw = self.dev = None
        self.samples = []
        try:
            import glob

            import torch
            p = torch.cuda.get_device_properties(device)
            want = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
            self.pci = want
            for d in sorted(glob.glob("/sys/class/drm/card*/device")):
                try:
                    ue = open(os.path.join(d, "uevent")).read()
                except OSError:
                    continue
                if f"PCI_SLOT_NAME={want}." in ue:
                    self.dev = d
                    hw = sorted(glob.glob(os.path.join(d, "hwmon", "hwmon*")))
                    self.hw = hw[0] if hw else None
                    break
        except Exception:   # noqa: BLE001 -- the state is reported, never fatal
            self.pci = None

    def _read(self, path, scale=1.0):
        try:
            return float(open(path).read().split()[0]) * scale
        except (OSError, ValueError, IndexError, TypeError):
            return None

    def sample(self):
        if not self.hw:
            return
        h = self.hw
        self.samples.append({"sclk_MHz": self._read(f"{h}/freq1_input", 1e-6),
                             "mclk_MHz": self._read(f"{h}/freq2_input", 1e-6),
                             "power_W": self._read(f"{h}/power1_input", 1e-6),
                             "junction_C": self._read(f"{h}/temp2_input", 1e-3),
                             "mem_C": self._read(f"{h}/temp3_input", 1e-3)})

    def report(self):
        if not self.dev:
            return {"pci": self.pci, "error": "no sysfs card with this PCI address"}
        out = {"pci": self.pci, "sysfs": self.dev, "samples": len(self.samples),
               "when": "after each timed repetition (hwmon short averages)"}
        for k in ("sclk_MHz", "mclk_MHz", "power_W", "junction_C", "mem_C"):
            v = sorted(s[k] for s in self.samples if s.get(k) is not None)
            if v:
                out[k] = {"min": round(v[0], 1), "median": round(v[len(v) // 2], 1),
                          "max": round(v[-1], 1)}
        out["power_cap_W"] = self._read(f"{self.hw}/power1_cap", 1e-6) if self.hw else None
        for f, key in (("pp_dpm_sclk", "sclk_levels"), ("pp_dpm_mclk", "mclk_levels"),
                       ("pp_dpm_fclk", "fclk_levels"), ("pp_dpm_socclk", "socclk_levels")):
            try:
                out[key] = open(os.path.join(self.dev, f)).read().split("\n")[:8]
                out[key] = [x.strip() for x in out[key] if x.strip()]
            except OSError:
                pass
        for f, key in (("power_dpm_force_performance_level", "perf_level"),
                       ("current_compute_partition", "compute_partition"),
                       ("current_memory_partition", "memory_partition")):
            try:
                out[key] = open(os.path.join(self.dev, f)).read().strip()
            except OSError:
                pass
        return out


MIN_ROWS_CANDIDATES = (128, 256, 512)   # dist_min_rows priced by the N > 1 warm-up
DEFAULT_MIN_ROWS = 256


def pricing_candidates(overlap_arg, min_rows_arg, N, rccl_check):
    """The (dist_min_rows, dist_overlap) pairs the N > 1 warm-up times (DESIGN.md
    section 6): overlap 0 / 1 / 2 (or the one given) x dist_min_rows 128 / 256
    (or the one given; auto prices them only up to N = 16384, where the
    replicated coarse tail is a large share of a rank's cycle).  A pair the
    RCCL self-check ran and did not pass bitwise is dropped (min_rows 16's
    check covers every overlap mode's exchanges; the candidates' own checks,
    "candidates" "<rows>:<overlap>", cover their partitions).  Never empty:
    falls back to (256, 0)."""
    ovs = [0, 1, 2] if overlap_arg == "auto" else [int(overlap_arg)]
    if min_rows_arg == "auto":
        rows = list(MIN_ROWS_CANDIDATES) if N <= 16384 else [DEFAULT_MIN_ROWS]
    else:
        rows = [int(min_rows_arg)]
    cands = []
    for r in rows:
        for ov in ovs:
            if rccl_check is not None:
                base = (rccl_check.get("modes") or {}).get(str(ov))
                own = (rccl_check.get("candidates") or {}).get(f"{r}:{ov}")
                if base is not None and not base.get("passed", False):
                    continue
                if own is not None and not own.get("passed", False):
                    continue
            cands.append((r, ov))
    return cands or [(DEFAULT_MIN_ROWS, 0)]


def price_partitions(mg, cur_rows, cands, make_ctx, barrier, max_over_ranks, set_overlap,
                     cycles=3):
    """Time `cycles` warm-up cycles (max over ranks) per (dist_min_rows,
    dist_overlap) candidate; a context is rebuilt (make_ctx(rows, 1)) only when
    the rows change -- rows descending, so the first is `mg`'s own when it was
    built with the largest -- and once more for the winner if needed.
    -> (context of the winner, its rows, best rows, best overlap,
    {"rows:overlap": ms per cycle})."""
    ab = {}
    for r in sorted({r for r, _ in cands}, reverse=True):
        if r != cur_rows:
            mg.close()
            mg = make_ctx(r, 1)
            cur_rows = r
        for rr, ov in cands:
            if rr != r:
                continue
            set_overlap(ov)
            mg.run_cycles(1)
            mg.synchronize()
            barrier()
            t0 = time.perf_counter()
            mg.run_cycles(cycles)
            mg.synchronize()
            ab[f"{r}:{ov}"] = round(max_over_ranks(time.perf_counter() - t0) / cycles * 1e3, 4)
    best_rows, best_ov = min(cands, key=lambda c: ab[f"{c[0]}:{c[1]}"])
    if best_rows != cur_rows:
        mg.close()
        mg = make_ctx(best_rows, 1)
        cur_rows = best_rows
    return mg, cur_rows, best_rows, best_ov, ab


class Watchdog:
    """A deadline on a phase that waits on the other ranks (N > 1): an RCCL hang
    would otherwise stall the run silently until an outer time limit.  On
    expiry: one error JSON line on stdout, then os._exit(1) (no exec, no GPU
    call from the timer thread)."""

    def __init__(self, phase, seconds, rank, world):
        self.phase, self.seconds, self.rank, self.world = phase, seconds, rank, world
        self.timer = None

    def _fire(self):
        print(json.dumps({"metric": "V-cycle grid-point-updates/sec at N=16384; achieved HBM "
                                    "GB/s vs peak", "value": None, "n_gpus": self.world,
                          "error": f"watchdog: phase '{self.phase}' exceeded "
                                   f"{self.seconds:.0f} s on rank {self.rank}"}), flush=True)
        sys.stderr.flush()
        os._exit(1)

    def __enter__(self):
        if self.world > 1 and self.seconds > 0:
            import threading
            self.timer = threading.Timer(self.seconds, self._fire)
            self.timer.daemon = True
            self.timer.start()
        return self

    def __exit__(self, *exc):
        if self.timer is not None:
            self.timer.cancel()
        return False


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
    def watch(phase):
        return Watchdog(phase, args.watchdog_s, rank, world)

    if world > 1:
        with watch("init_process_group"):
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if world > 1:
            dist.barrier()

    N, L = args.N, args.levels
    if args.weak and world > 1:
        # points per GPU ~ constant: N grows by 2 per 4x ranks (power of two)
        g = 1
        while 4 * g <= world:
            N, L, g = 2 * N, L + 1, 4 * g
    # the (dist_min_rows, dist_overlap) pairs the warm-up may price
    cand_rows = sorted({r for r, _ in pricing_candidates(args.overlap, args.min_rows, N, None)})

    rccl_check = None
    if world > 1 and args.rccl_check:
        # libmgx's own RCCL transport with real peers vs a one-GPU context,
        # bitwise (small problem, before and outside the timed region), also
        # for every partition candidate
        from hpcclassmultigridproject_amd import dist as mgdist
        with watch("rccl_selfcheck"):
            rccl_check = mgdist.rccl_selfcheck(world, rank, local, min_rows=cand_rows,
                                               candidate_fp=args.fp_mode)

    nu = -4e-4
    dt = 1.0 / N / 10
    fp = _lib.FP_FMA if args.fp_mode == "fma" else _lib.FP_BITWISE
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

    def make_ctx(min_rows, warmup):
        """The bench context: created (row-partitioned over the ranks with
        dist_min_rows = min_rows when N > 1), uploaded, rhs formed and
        `warmup` untimed cycles run."""
        dist_kw = {}
        if world > 1:
            from hpcclassmultigridproject_amd import dist as mgdist
            _lib.set_tuning("dist_min_rows", min_rows)
            dist_kw = dict(world=world, rank=rank, unique_id=mgdist.broadcast_unique_id())
        m = pkg.Multigrid(N, L, dt, nu, nsmooth=args.nsmooth, device=local,
                          smoother=args.smoother, fuse=args.fuse, tower_mode=tower, fp_mode=fp,
                          **dist_kw)
        if row_upload:
            lo, hi = m.dist_rows(0)
            m.upload_rows([pkg.init_problem_rows(N, lo, hi + 1, nthreads=16)])
        else:
            u0, v1, v2 = pkg.init_problem(N, nthreads=16)
            m.upload(u0, v1, v2)
            del u0, v1, v2
        m.rhs()
        for _ in range(warmup):
            m.run_cycles(1)
        m.synchronize()
        return m

    setup_wd = watch("set-up (context, upload, warm-up)").__enter__()
    cands = pricing_candidates(args.overlap, args.min_rows, N, rccl_check)
    cur_rows = cands[-1][0] if world > 1 else None
    mg = make_ctx(cur_rows, args.warmup)
    setup_wd.__exit__(None, None, None)

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    overlap_ab = None
    if world > 1:
        # price the partition and exchange schedules on this machine (untimed
        # warm-up): the early level-0 exchange behind the coarse levels pays
        # over xGMI but not on one GPU's virtual ranks, and dist_min_rows 128
        # partitions one level more (less replicated tail, one more RCCL
        # exchange per cycle); only pairs whose RCCL
        # self-check passed bitwise are candidates
        if len(cands) > 1:
            with watch("partition / overlap pricing"):
                mg, cur_rows, best_rows, best_ov, overlap_ab = price_partitions(
                    mg, cur_rows, cands, make_ctx, barrier, max_over_ranks,
                    lambda ov: _lib.set_tuning("dist_overlap", ov))
        else:
            best_rows, best_ov = cands[0]
        _lib.set_tuning("dist_overlap", best_ov)
        mg.run_cycles(1)
        mg.synchronize()
    la = mg.dist_info()[2]

    gpu_state = GpuState(local)

    def timed_reps(m, reps, prof, state=None):
        """SURVEY 8(d) protocol: `reps` repetitions of K cycles, each bracketed
        by barrier + synchronize, max over ranks; HIP events around the
        finest-level launches (prof); the GPU's clocks sampled after each
        (state); -> (seconds per repetition, residual)."""
        m.profile_reset()
        if prof:
            # events around the finest-level launches only (the dominant
            # kernels); events around every small-level launch would cost ~7%
            m.profile(True, finest_only=True)
        secs, res = [], None
        for _ in range(reps):
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            # K steps = K V-cycles, each followed by its residual norm (read
            # back per cycle, as mg_outer does); the K-th cycle's solution is
            # materialised
            res = m.run_cycles(args.steps)
            m.synchronize()
            barrier()
            torch.cuda.synchronize()
            secs.append(max_over_ranks(time.perf_counter() - t0))
            if state is not None:
                state.sample()
        return secs, res

    def dominant(m):
        """(kind, level 0, launches, ms, canonical bytes, compulsory bytes) of
        the finest-level kernel with the largest device time since the reset."""
        best = None
        for kind in _lib.KERNEL_NAMES:
            n, ms, b, cb = m.profile_get_ex(kind, 0)
            if n and (best is None or ms > best[3]):
                best = (kind, 0, n, ms, b, cb)
        return best

    with watch("timed region"):
        rep_s, res = timed_reps(mg, args.reps, not args.no_profile, gpu_state)
    elapsed = sorted(rep_s)[len(rep_s) // 2]   # the median repetition
    best = dominant(mg)
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
    pcie = None
    if world == 1 and not row_upload:
        # the boundary's host-buffer rate (never `value`): the same K cycles
        # with the host arrays handed over before (mgx_upload: H2D copies +
        # the device-built tower + the upload-time velocity checks) and the
        # solution copied back after, inside the clock
        u0, v1, v2 = pkg.init_problem(N, nthreads=16)
        uo = np.empty_like(u0)
        mg.synchronize()
        t0 = time.perf_counter()
        mg.upload(u0, v1, v2)
        mg.synchronize()
        t_up = time.perf_counter() - t0
        mg.rhs()
        t1 = time.perf_counter()
        mg.run_cycles(args.steps)
        mg.synchronize()
        t_cyc = time.perf_counter() - t1
        t2 = time.perf_counter()
        mg.download(uo)
        t_down = time.perf_counter() - t2
        del u0, v1, v2, uo
        pcie = {"upload_s": round(t_up, 4), "cycles_s": round(t_cyc, 5),
                "download_s": round(t_down, 4),
                "value_incl": (N - 1) ** 2 * args.steps / (t_up + t_cyc + t_down),
                "note": f"{args.steps} V-cycles with mgx_upload (3 host arrays of "
                        f"{(N + 1) ** 2 * 8 / 1e9:.2f} GB: H2D + tower + velocity checks) "
                        f"before and mgx_download after, inside the clock; the bench value "
                        f"starts with the inputs resident in HBM"}
    mg.close()

    def roofline(best, mode, v_extra=0.0):
        """Roofline of the dominant kernel: achieved = its compulsory bytes per
        launch (each array the fused pass must read or write, once) / its live
        mean event duration; v_extra: bytes of the 2-D velocity arrays the pass
        reads on the generic path (already in its compulsory bytes there)."""
        kind, lvl, n0, ms0, b0, cb0 = best
        per_launch = cb0 / n0
        avg_s = ms0 * 1e-3 / n0
        achieved = per_launch / avg_s / 1e9
        r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
             "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
             "kernel": f"{_lib.KERNEL_NAMES[kind]} level {lvl}",
             "compulsory_bytes_per_launch": per_launch,
             "avg_launch_ms": round(avg_s * 1e3, 4),
             "launches": n0,
             "canonical_bytes_per_launch": b0 / n0,
             "canonical_equiv_GBs": round(b0 / n0 / avg_s / 1e9, 1)}
        # the committed PMC traffic is per launch of the single-GPU pass; a
        # rank's row block moves a fraction of it, so it is not reused there
        ids = KERNEL_IDS.get((mode, kind)) if (N, L, args.nsmooth, args.smoother, args.fuse,
                                                world) == (16384, 9, 3, 0, 3, 1) else None
        if not ids:
            r["traffic_null_reason"] = "no committed PMC profile for this configuration"
            return r
        kname, traffic, tsrc = lookup_traffic(ids, mode)
        if not traffic:
            r["traffic_null_reason"] = tsrc
            return r
        r["kernel"] += f" = {kname}"
        r["traffic"] = traffic
        r["traffic_source"] = tsrc
        r["traffic_over_compulsory"] = round(traffic / per_launch, 3)
        # the profile's own kernel durations (rocprofv3, sum of the pass's
        # launches): the live event mean should agree with them.  The HBM
        # rate is the profile's bytes over the profile's own durations (one
        # box, one run), never the PMC bytes of one box over another's clock
        _, pms, _ = lookup_traffic(ids, mode, "ms_profiled")
        if pms:
            r["profiled_launch_ms"] = round(pms, 4)
            r["live_over_profiled"] = round(avg_s * 1e3 / pms, 4)
            r["hbm_GBs"] = round(traffic / (pms * 1e-3) / 1e9, 1)
            r["hbm_frac"] = round(r["hbm_GBs"] / HBM_PEAK_GBS, 4)
            r["hbm_note"] = ("hbm_GBs = PMC bytes / rocprof duration of the same profile run "
                             "(traffic_source); achieved = compulsory bytes / this run's live "
                             "HIP-event mean")
        # VALU wave-instructions per launch (PMC SQ_INSTS_VALU, same profile)
        # against the issue capacity of the live duration (one wave64
        # instruction per 4 cycles per SIMD, 1024 SIMDs, 2.4 GHz peak clock:
        # a lower bound on the busy fraction)
        _, valu, _ = lookup_traffic(ids, mode, "SQ_INSTS_VALU")
        if valu:
            cap = 1024 * avg_s * 2.4e9 / 4
            r["valu"] = {"insts_per_launch": valu, "issue_capacity": round(cap),
                         "issue_frac": round(valu / cap, 4),
                         "note": "VALU wave-instructions / (1024 SIMDs x 2.4 GHz / 4 "
                                 "cycles per wave64 op x live mean duration)"}
        return r

    def side_run(label, fpm, tuning, reps, tower_mode=None):
        """The same workload in another configuration (one GPU): fp_mode fpm,
        process tuning keys `tuning` and velocity tower `tower_mode` (default:
        the headline's), `reps` repetitions of K cycles."""
        keys = {k: _lib.get_tuning(k) for k in tuning}
        try:
            for k, v in tuning.items():
                _lib.set_tuning(k, v)
            g = pkg.Multigrid(N, L, dt, nu, nsmooth=args.nsmooth, device=local,
                              smoother=args.smoother, fuse=args.fuse,
                              tower_mode=tower if tower_mode is None else tower_mode,
                              fp_mode=fpm)
            u0, v1, v2 = pkg.init_problem(N, nthreads=16)
            g.upload(u0, v1, v2)
            del u0, v1, v2
            g.rhs()
            g.run_cycles(2)
            g.synchronize()
            secs, _ = timed_reps(g, reps, True)
            b = dominant(g)
            g.profile(False)
            g.close()
        finally:
            for k, v in keys.items():
                _lib.set_tuning(k, v)
        med = sorted(secs)[len(secs) // 2]
        mode = ("fma" if fpm == _lib.FP_FMA else "bitwise") + \
               ("-generic" if tuning.get("sep_velocity") == 0 else "")
        return {"label": label, "ms_per_step": round(med / args.steps * 1e3, 4),
                "rep_ms_per_step": [round(x / args.steps * 1e3, 4) for x in secs],
                "value": (N - 1) ** 2 * args.steps / med,
                "roofline": roofline(b, mode) if b else None}

    fp_name = "fma" if fp == _lib.FP_FMA else "bitwise"
    other = None
    generic = None
    nonrank1 = None
    correct = None
    if world == 1 and not args.no_compare:
        # the other arithmetic mode (bitwise: every value the reference's)
        ofp = _lib.FP_BITWISE if fp == _lib.FP_FMA else _lib.FP_FMA
        other = side_run("bitwise" if ofp == _lib.FP_BITWISE else "fma", ofp, {}, 3)
        # the generic velocity path (2-D v1 / v2 on every row of every level:
        # sep_velocity = zero_rows = 0, hence no generator either): the
        # headline reads the reference flow's exact rank-1 factors on level 0,
        # regenerates levels 1-2's velocity from them (vgen) and skips the
        # coarser levels' all-zero velocity rows
        generic = side_run("generic velocity", fp, {"sep_velocity": 0, "zero_rows": 0}, 3)
        generic["note"] = "sep_velocity=0, zero_rows=0: every velocity row read from HBM"
        # a velocity field that is not an exact rank-1 product (any user
        # field): no factors, so no generator either, but the reference
        # tower's all-zero coarse rows (whatever the field) still
        # come from the zero row -- what such a field runs at
        nonrank1 = side_run("non-rank-1 velocity field", fp, {"sep_velocity": 0}, 3)
        nonrank1["note"] = ("sep_velocity=0 (factors and vgen off); zero_rows on: the "
                            "reference tower's zero coarse rows hold for any field")
        if tower == pkg._lib.TOWER_REFERENCE:
            # the correct velocity tower (SURVEY K2's fix; what every row-block
            # and N > 16384 run uses): levels 1..L-2 generate their velocity
            # from the finest factors (strided vgen), no all-zero coarse rows;
            # parity: tests/test_gpu_solver.py::test_vcycle_correct_tower_vs_reference
            correct = side_run("correct tower", fp, {}, 3, tower_mode=pkg._lib.TOWER_CORRECT)
            correct["note"] = ("TOWER_CORRECT: every coarse velocity level injected from the "
                               "one above; bitwise the compiled reference's mg_inner on that "
                               "tower at N=16384 (sha256 fixture)")

    roof = roofline(best, fp_name) if best else None
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
        # the velocity factors regenerate them bitwise instead of reading them.
        # An equivalent rate only -- no kernel moved these bytes, so no fraction
        vb = 2.0 * 8.0 * (N + 1) * ((N + 1 + 15) // 16 * 16)
        a2 = (roof["compulsory_bytes_per_launch"] + vb) / (roof["avg_launch_ms"] * 1e-3) / 1e9
        roof["algorithmic_2d_velocity"] = {
            "bytes_per_launch": roof["compulsory_bytes_per_launch"] + vb,
            "equiv_GBs": round(a2, 1),
            "note": "compulsory bytes with v1, v2 counted as read (they are regenerated "
                    "bitwise from their rank-1 factors instead, not moved)"}
    reps_ms = [x / args.steps * 1e3 for x in rep_s]
    out = {
        "metric": f"V-cycle grid-point-updates/sec at N={N}; achieved HBM GB/s vs peak",
        "value": value, "unit": "grid-point-updates/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "reps": len(rep_s), "median": value,
        "rep_ms_per_step": [round(x, 4) for x in reps_ms],
        "spread": {"min_ms_per_step": round(min(reps_ms), 4),
                   "max_ms_per_step": round(max(reps_ms), 4),
                   "rel": round((max(reps_ms) - min(reps_ms)) / (elapsed / args.steps * 1e3), 4)},
        "smoother_point_updates_per_s": smoother_pts * args.steps / elapsed,
        "scaling": "single" if world == 1 else ("weak" if args.weak else "strong"),
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: the reference problem (Gaussian u0, rotating velocity), "
                "generated on the host with glibc libm",
        "config": {"workload": f"N={N} fp64 V-cycle, L={L} (coarsest {N >> (L - 1)}), "
                               f"nu_smooth={args.nsmooth}, + residual/norm per step",
                   "N": N, "levels": L, "nsmooth": args.nsmooth,
                   "fp_mode": fp_name,
                   "parity": ("fma: contracted smoothing passes, max|duT| <= 1e-12 vs the "
                              "reference with identical cycle counts (tests/test_gpu_fma.py)"
                              if fp == _lib.FP_FMA else
                              "bitwise: u equal to the reference bit for bit "
                              "(tests/test_gpu_solver.py sha256)"),
                   "protocol": f"{args.warmup} warm-up cycles, then {len(rep_s)} repetitions "
                               f"of {args.steps} timed cycles; value = the median repetition "
                               "(SURVEY 8(d))",
                   "tower": ("correct (row-block upload)" if row_upload else
                             "correct" if tower == pkg._lib.TOWER_CORRECT else "reference"),
                   "parallelism": (f"row-partition x{world} on levels 0..{la - 1}, "
                                   f"levels {la}..{L - 1} replicated" if world > 1
                                   else "single"),
                   "dist_overlap": _lib.get_tuning("dist_overlap") if world > 1 else None,
                   "dist_min_rows": cur_rows,
                   "pricing_ms_per_cycle": overlap_ab,
                   "pricing_note": ("warm-up cycles per '<dist_min_rows>:<dist_overlap>' "
                                    "candidate, max over ranks; the fastest is timed")
                   if overlap_ab else None,
                   "last_residual": res},
        "roofline": roof,
        "gpu_state": gpu_state.report(),
        "kernels": kernels,
        "velocity": velocity_note(fac.value, tower == pkg._lib.TOWER_CORRECT, L)
                    if world == 1 else None,
        "other_fp_mode": other,
        "generic_velocity_path": generic,
        "non_rank1_velocity": nonrank1,
        "correct_tower": correct,
    }
    # what the loaded library was built from (csrc/Makefile stamps it): the
    # traffic lookup above used its kernel sha, not the tree's
    bid = _lib.build_id()
    bid["matches_tree"] = bid["kernel_sources_sha256"] == kernels_sha()
    out["build"] = bid
    if other is not None:   # the reference's bits, the library default, beside the headline
        out["value_bitwise" if fp == _lib.FP_FMA else "value_fma"] = other["value"]
    if pcie is not None:
        out["host_buffers"] = pcie
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
