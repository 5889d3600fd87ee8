#!/bin/bash
# PMC passes for the V-cycle kernels (one counter group per rocprofv3 run, as
# MI355X_MICROARCH.md prescribes).  Usage: tools/pmc_collect.sh OUTDIR [N L cycles]
set -e
OUT=${1:-gpurun_out/pmc}
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
CGROUPS=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
  "GRBM_GUI_ACTIVE GRBM_COUNT"
)
# PMC_GROUPS="grp1;grp2" overrides the list
if [ -n "$PMC_GROUPS" ]; then IFS=';' read -r -a CGROUPS <<< "$PMC_GROUPS"; fi
for grp in "${CGROUPS[@]}"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/$tag" -o run --output-format csv -- python3 tools/pmc_vcycle.py "$@" > "$OUT/$tag.log" 2>&1 || echo "group $tag failed"
done
