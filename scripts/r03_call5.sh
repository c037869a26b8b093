# GPU box: GPU parity suite, C5/C2 bench (+ rocprof of C5), dense phase clocks with ablations,
# then the H2D breakdown.  Each GPU step under its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-c5x}
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_gpu_$T.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu_$T.log | head -30; exit $rc; }
fi
TAG=$T PROF=1 WLS="${WLS:-c5 c2}" bash scripts/bench_all.sh || exit 1
timeout -k 10 300 python -u scripts/prof_dense.py c5 ${ABL:-0,16,32} > gpurun_out/${T}_prof_dense.txt 2>&1 || { tail -5 gpurun_out/${T}_prof_dense.txt; exit 1; }
cat gpurun_out/${T}_prof_dense.txt
timeout -k 10 300 python -u scripts/h2d_time.py c5 > gpurun_out/${T}_h2d.txt 2>&1 || { tail -5 gpurun_out/${T}_h2d.txt; exit 1; }
cat gpurun_out/${T}_h2d.txt
echo R03_CALL5_DONE
