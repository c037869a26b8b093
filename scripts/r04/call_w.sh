# round 4: k_tile_dense deletion reads' 2nd / 3rd op words read with the first, before the walk
# loop — GPU suite, A/B of the C5 line against the previous build (four rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4w_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4w_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4w_pytest_gpu.log
WL=c5 TAG=abw1 LIBS="libs2c_prev.so libs2c.so" bash scripts/ab_libs.sh || exit 1
WL=c5 TAG=abw2 LIBS="libs2c.so libs2c_prev.so" bash scripts/ab_libs.sh || exit 1
