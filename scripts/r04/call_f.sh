# round 4: k_tile coverage differences combined over equal neighbours — GPU tests, A/B on C4 / C3,
# PMC of C4 (LDS conflicts)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
NOTEST= TPS=0 bash scripts/gpu_iter.sh || exit 1
WL=c4 TAG=abf4 LIBS="libs2c.so libs2c_prev.so" bash scripts/ab_libs.sh || exit 1
WL=c3 TAG=abf3 LIBS="libs2c.so libs2c_prev.so" bash scripts/ab_libs.sh || exit 1
NOTEST=1 PMC=1 WL=c4 bash scripts/gpu_iter.sh || exit 1
