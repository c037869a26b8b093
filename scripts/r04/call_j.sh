# round 4: C5 dense kernel VALU / LDS per ablated phase on the closing build (prof variant)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
ABLS="0 2 4 8 32 62" WL=c5 bash scripts/pmc_abl_dense.sh > gpurun_out/r4j_abl_c5.txt 2>&1 || { tail -20 gpurun_out/r4j_abl_c5.txt; exit 1; }
cat gpurun_out/r4j_abl_c5.txt
