# One iteration on the GPU box: parity tests, then C5 bench at the planner's tile width and at
# forced widths (S2C_TILE_POS), each step under its own time limit; the first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
fi
for tp in ${TPS:-0}; do
  if [ "$tp" = 0 ]; then unset S2C_TILE_POS; else export S2C_TILE_POS=$tp; fi
  timeout -k 10 300 python -u bench.py --workload ${WL:-c5} --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/it_$tp.json 2> gpurun_out/it_$tp.err || { tail -5 gpurun_out/it_$tp.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/it_$tp.json'));print('tp', $tp, 'step', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, d['parity'])"
done
if [ -n "$PROF" ]; then
  timeout -k 10 300 python -u scripts/prof_dense.py ${WL:-c5} 0 > gpurun_out/prof_dense.txt 2>&1; rc=$?; cat gpurun_out/prof_dense.txt; [ $rc -eq 0 ] || exit $rc
  bash scripts/pmc_ablate_dense.sh > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
  echo PMC_OK
fi
if [ -n "$PMC" ]; then   # VALU / LDS instructions and LDS conflicts of the workload's tile kernels
  cd /tmp
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
      SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_it_${WL:-c5} -o run \
      -- python3 $GRAFT_REPO_ROOT/bench.py --workload ${WL:-c5} --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-file-parse \
      > $GRAFT_REPO_ROOT/gpurun_out/pmc_it.log 2>&1 || { echo "pmc failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc_it.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  python3 scripts/pmc_summary.py gpurun_out/pmc_it_${WL:-c5} k_tile | grep -E "VALU|LDS|WAVES|duration"
fi
