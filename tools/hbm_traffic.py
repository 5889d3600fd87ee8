"""Per-kernel HBM traffic from a pmc_summary.py JSON (tools/pmc_collect.sh run).
    python tools/hbm_traffic.py gpurun_out/pmc.json > profiles/<round>_hbm_traffic.json
hbm_read_bytes = 2 x FETCH_SIZE KiB (gfx950 FETCH_SIZE counts half of a
16-B/lane streaming read, MI355X_MICROARCH.md HBM section); hbm_write_bytes =
WRITE_SIZE KiB (exact for 16-B/lane streaming stores).  Means per dispatch."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import kernels_sha, loaded_kernels_sha  # noqa: E402  (kernel sources sha256)

src = json.load(open(sys.argv[1]))
out = {"note": "rocprofv3 --pmc, one counter group per run (tools/pmc_collect.sh), "
               "N=16384 L=9, mean per dispatch; hbm_read_bytes = 2 x FETCH_SIZE KiB "
               "(gfx950 FETCH_SIZE counts half of a 16-B/lane streaming read, "
               "MI355X_MICROARCH.md HBM); hbm_write_bytes = WRITE_SIZE KiB",
       # bench.py uses these bytes only with a library built from these kernel
       # sources (mgx_build_id of the library that was profiled, = the tree's)
       "kernel_sources_sha256": loaded_kernels_sha(),
       "tree_kernel_sources_sha256": kernels_sha(),
       "mode": os.environ.get("MGX_PMC_MODE", "fma"),
       "kernels": {}}
for k, v in src.items():
    if "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
        continue
    rd = 2.0 * v["FETCH_SIZE"] * 1024
    wr = v["WRITE_SIZE"] * 1024
    e = {"hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes": rd + wr,
         "ms_profiled": v.get("ms"), "dispatches": v.get("dispatches")}
    if v.get("ms"):
        e["hbm_TBs_profiled"] = (rd + wr) / (v["ms"] * 1e-3) / 1e12
    cyc = v.get("SQ_WAVE_CYCLES")
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if cyc and c in v:
            e[c + "_frac"] = v[c] / cyc
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT"):
        if c in v:
            e[c] = v[c]
    out["kernels"][k] = e
print(json.dumps(out, indent=1))
