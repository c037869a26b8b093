# round 4: k_tile coverage ends summed per lane in registers (one LDS atomic per change of
# position) — GPU suite, then A/B against the previous build on C4, C3 and C2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4v_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4v_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4v_pytest_gpu.log
WL=c4 TAG=abcv4a LIBS="libs2c_prev.so libs2c.so" bash scripts/ab_libs.sh || exit 1
WL=c4 TAG=abcv4b LIBS="libs2c.so libs2c_prev.so" bash scripts/ab_libs.sh || exit 1
WL=c3 TAG=abcv3 LIBS="libs2c_prev.so libs2c.so" bash scripts/ab_libs.sh || exit 1
WL=c2 TAG=abcv2 LIBS="libs2c_prev.so libs2c.so" bash scripts/ab_libs.sh || exit 1
