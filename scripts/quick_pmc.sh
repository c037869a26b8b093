set -o pipefail
cd $GRAFT_REPO_ROOT
WLS="c5 c5nd" bash scripts/gpu_quick.sh || exit $?
bash scripts/pmc_busy.sh > /dev/null 2>&1 || { echo pmc fail; exit 1; }
echo PMC_OK
