set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 bash tools/ab_libs.sh 3 --fp fma > gpurun_out/r4m_ablibs.log 2>&1 || exit $?
cat gpurun_out/r4m_ablibs.log
