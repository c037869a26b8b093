# round 4: k_tile_dense without the workgroup barrier between the fast walk and the queued
# walks (each wave's queued work is its own) — GPU suite, A/B of the C5 line (four rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4z_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4z_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4z_pytest_gpu.log
WL=c5 TAG=abz1 LIBS="libs2c_prev.so libs2c.so" bash scripts/ab_libs.sh || exit 1
WL=c5 TAG=abz2 LIBS="libs2c.so libs2c_prev.so" bash scripts/ab_libs.sh || exit 1
