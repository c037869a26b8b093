# round 4: dense count in 4 planes when no lane's count can reach 16 — GPU parity suite
# (dense / golden tests), then A/B of the C5 line against the previous build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4m_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4m_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4m_pytest_gpu.log
WL=c5 TAG=abnb LIBS="libs2c_prev.so libs2c.so" bash scripts/ab_libs.sh || exit 1
