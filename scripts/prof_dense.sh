set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/prof_dense.py c5 0 > gpurun_out/prof_dense.txt 2>&1; rc=$?; cat gpurun_out/prof_dense.txt; exit $rc
