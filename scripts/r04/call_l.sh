# round 4: C5 dense kernel with the one-at-a-time slow votes left out (ablation 64)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
ABLS="64 0" WL=c5 bash scripts/pmc_abl_dense.sh > gpurun_out/r4l_abl_c5.txt 2>&1 || { tail -20 gpurun_out/r4l_abl_c5.txt; exit 1; }
cat gpurun_out/r4l_abl_c5.txt
