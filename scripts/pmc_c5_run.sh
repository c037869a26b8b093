set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/prof_dense.py c5 0,4,2,8,6 > gpurun_out/prof_dense_c5.txt 2>&1; rc=$?; cat gpurun_out/prof_dense_c5.txt; [ $rc -eq 0 ] || exit $rc
WL=c5 timeout -k 10 900 bash scripts/pmc.sh
