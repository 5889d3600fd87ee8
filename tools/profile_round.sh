#!/bin/bash
# Profiles for one round, written to gpurun_out/prof_<tag>/ (copy to profiles/):
#   kernel_stats.csv  rocprofv3 --kernel-trace --stats of the default bench
#   bench.json        the bench line of that run
#   pmc.json          PMC counters per kernel (separate passes, tools/pmc_collect.sh)
#   hbm_traffic.json  HBM bytes per dispatch derived from pmc.json
# Usage (on the GPU box): bash tools/profile_round.sh TAG
set -e
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off --no-generic > "$OUT/bench_prof.log" 2>&1
grep '^{' "$OUT/bench_prof.log" | tail -1 > "$OUT/bench.json"
cp "$(find "$OUT/trace" -name 'run_kernel_stats.csv' | head -1)" "$OUT/kernel_stats.csv"
# same cycle pattern as the bench: one run_cycles(10) call
bash tools/pmc_collect.sh "$OUT/pmc" 16384 9 10
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc.json"
python3 tools/hbm_traffic.py "$OUT/pmc.json" > "$OUT/hbm_traffic.json"
rm -rf "$OUT/trace" "$OUT/pmc"
