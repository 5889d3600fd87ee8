#!/bin/bash
# Profiles for one round, written to gpurun_out/prof_<tag>/ (copy to profiles/):
#   kernel_stats.csv  rocprofv3 --kernel-trace --stats of the default bench
#   bench.json        the bench line of that run
#   pmc_<mode>.json          PMC counters per kernel (separate passes, tools/pmc_collect.sh)
#   hbm_traffic_<mode>.json  HBM bytes per dispatch derived from it
#   (mode: fma, bitwise, fma-generic; bench.py picks the file of its mode)
# Usage (on the GPU box): bash tools/profile_round.sh TAG
set -e
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --reps 3 --cpu-baseline off --no-compare > "$OUT/bench_prof.log" 2>&1
grep '^{' "$OUT/bench_prof.log" | tail -1 > "$OUT/bench.json"
cp "$(find "$OUT/trace" -name 'run_kernel_stats.csv' | head -1)" "$OUT/kernel_stats.csv"
rm -rf "$OUT/trace"
# PMC per arithmetic mode, the bench's cycle pattern (one run_cycles(10) call):
# fma (the headline), bitwise, fma on the generic velocity path
for mode in fma bitwise fma-generic; do
  fp=${mode%-generic}
  gen=0; [ "$mode" = "fma-generic" ] && gen=1
  bash tools/pmc_collect.sh "$OUT/pmc_$mode" 16384 9 10 $fp $gen
  python3 tools/pmc_summary.py "$OUT/pmc_$mode" > "$OUT/pmc_$mode.json"
  MGX_PMC_MODE=$mode python3 tools/hbm_traffic.py "$OUT/pmc_$mode.json" > "$OUT/hbm_traffic_$mode.json"
  rm -rf "$OUT/pmc_$mode"
done
