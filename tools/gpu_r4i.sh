set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4i
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4i/re0 -o run --output-format csv -- python3 tools/ab_levels.py xre=0 --fp fma --rounds 1 --cycles 5 > gpurun_out/r4i/re0.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4i/re1 -o run --output-format csv -- python3 tools/ab_levels.py xre=1 --fp fma --rounds 1 --cycles 5 > gpurun_out/r4i/re1.log 2>&1 || exit $?
python3 tools/kgrid.py gpurun_out/r4i/re0 smooth > gpurun_out/r4i/re0.txt
python3 tools/kgrid.py gpurun_out/r4i/re1 smooth > gpurun_out/r4i/re1.txt
head -12 gpurun_out/r4i/re0.txt gpurun_out/r4i/re1.txt
