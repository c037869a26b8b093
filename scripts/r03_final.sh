# GPU box, the round's closing evidence: the GPU parity suite, the default bench line
# (C5, cpu_baseline legs, file parse), the same command under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-fin}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_$T.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu_$T.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -5 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_default -o out -- python3 bench.py \
  > gpurun_out/prof_${T}_default.log 2>&1 || { tail -5 gpurun_out/prof_${T}_default.log; exit 1; }
echo R03_FINAL_DONE
