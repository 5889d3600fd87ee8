set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 bash tools/profile_round.sh r4a > gpurun_out/r4e_prof.log 2>&1
rc=$?
tail -5 gpurun_out/r4e_prof.log
ls gpurun_out/prof_r4a
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tools/ab_libs.sh 3 --fp fma > gpurun_out/r4e_ablibs.log 2>&1
tail -12 gpurun_out/r4e_ablibs.log
