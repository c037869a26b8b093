# round 4: k_tile_dense '-' runs added a word at a time (8 row increments per word) instead of
# position by position at their ends — GPU suite, A/B of the C5 line, phase clocks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4s_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4s_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4s_pytest_gpu.log
WL=c5 TAG=abcr1 LIBS="libs2c_prev.so libs2c.so" bash scripts/ab_libs.sh || exit 1
WL=c5 TAG=abcr2 LIBS="libs2c.so libs2c_prev.so" bash scripts/ab_libs.sh || exit 1
S2C_LIB=libs2c_prof.so timeout -k 10 300 python -u scripts/prof_dense.py c5 0 > gpurun_out/r4s_dense_phases_c5.txt 2>&1 || { tail -20 gpurun_out/r4s_dense_phases_c5.txt; exit 1; }
cat gpurun_out/r4s_dense_phases_c5.txt
