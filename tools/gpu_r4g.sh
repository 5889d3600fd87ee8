set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/rccl_selfcheck1.py > gpurun_out/r4g_rccl1.log 2>&1 || exit $?
tail -2 gpurun_out/r4g_rccl1.log
timeout -k 10 500 bash tools/ab_libs.sh 3 --fp fma > gpurun_out/r4g_ablibs.log 2>&1 || exit $?
tail -12 gpurun_out/r4g_ablibs.log
