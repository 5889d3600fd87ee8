"""Per-kernel resource usage of the stencil kernels (VGPRs, spills, LDS,
occupancy) from hipcc's -Rpass-analysis=kernel-resource-usage remarks.
    python tools/kres.py [filter] [extra -D flags...]
The source file follows the filter: xsmooth / xtile -> xsmooth.hip, wsmooth /
smooth_tile -> wsmooth.hip, else kernels.hip; MGX_KRES_DIR overrides the
source directory (e.g. an older checkout)."""
import os
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else "xsmooth"
src = ("xsmooth.hip" if ("xsmooth" in flt or "xtile" in flt) else
       "wsmooth.hip" if ("wsmooth" in flt or "smooth_tile" in flt) else "kernels.hip")
srcdir = os.environ.get("MGX_KRES_DIR", "hpcclassmultigridproject_amd/csrc")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
       "-ffp-contract=off", "-fno-fast-math", "-Wno-pass-failed", "--cuda-device-only", "-c",
       "-o", "/tmp/kres.o", os.path.join(srcdir, src),
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        cur = re.sub(r"\(.*", "", dm.replace("(anonymous namespace)::", "")).replace("mgx::", "")
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for k, v in rows.items():
    if flt in k:
        print(f"{k:55s} VGPR {v.get('VGPRs'):>4} AGPR {v.get('AGPRs'):>3} vspill "
              f"{v.get('VGPRs Spill'):>3} sspill {v.get('SGPRs Spill'):>3} LDS "
              f"{v.get('LDS Size [bytes/block]'):>6} occ {v.get('Occupancy [waves/SIMD]')}")
