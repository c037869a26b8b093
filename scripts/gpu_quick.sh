# quick iteration: dense-path GPU tests, C5 (and C5 without -d) bench, phase clocks
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-dense or c5 or hip_path or batch_model}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
for wl in ${WLS:-c5}; do
for tp in ${TPS:-0}; do
  if [ "$tp" = 0 ]; then unset S2C_TILE_POS; else export S2C_TILE_POS=$tp; fi
  timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-file-parse > gpurun_out/q_$wl.json 2> gpurun_out/q_$wl.err || { tail -5 gpurun_out/q_$wl.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/q_$wl.json'));print('$wl tp $tp step', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, d['parity'])"
done
done
unset S2C_TILE_POS
if [ -n "$PROF" ]; then
timeout -k 10 300 python -u scripts/prof_dense.py c5 0 > gpurun_out/prof_dense.txt 2>&1; rc=$?; tail -9 gpurun_out/prof_dense.txt; exit $rc
fi
