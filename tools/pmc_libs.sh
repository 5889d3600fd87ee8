#!/bin/bash
# PMC comparison of libmgx variants: for the default libmgx.so and every
# libmgx_<name>.so, the SQ instruction / wait counters of one V-cycle run
# (tools/pmc_collect.sh groups 3-4) -> gpurun_out/pmclibs/<variant>.json
#   bash tools/pmc_libs.sh [N L cycles]
set -e
O=gpurun_out/pmclibs; mkdir -p $O
for lib in hpcclassmultigridproject_amd/libmgx.so hpcclassmultigridproject_amd/libmgx_*.so; do
  [ -f "$lib" ] || continue
  v=$(basename $lib .so)
  MGX_LIB=$lib PMC_GROUPS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
    bash tools/pmc_collect.sh $O/raw_$v "$@"
  python3 tools/pmc_summary.py $O/raw_$v > $O/$v.json
  rm -rf $O/raw_$v
  echo "$v done"
done
