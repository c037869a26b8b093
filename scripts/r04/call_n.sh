# round 4: VALU of the dense kernel with the 4-plane count (prof build, one PMC pass)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
ABLS="0" WL=c5 bash scripts/pmc_abl_dense.sh > gpurun_out/r4n_pmc_c5.txt 2>&1 || { tail -20 gpurun_out/r4n_pmc_c5.txt; exit 1; }
cat gpurun_out/r4n_pmc_c5.txt
