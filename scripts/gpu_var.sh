# quick experiment: dense-path GPU tests on libs2c.so, then the C5 bench on libs2c.so and on
# each variant library (VARS="occ4 ..." → sam2consensus_amd/libs2c_<v>.so, `make variant`)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-dense or c5 or hip_path or batch_model or kat or fuzz}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
fi
for wl in ${WLS:-c5}; do
for v in base ${VARS}; do
  if [ "$v" = base ]; then unset S2C_LIB; else export S2C_LIB=libs2c_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-file-parse > gpurun_out/v_${wl}_$v.json 2> gpurun_out/v_${wl}_$v.err || { tail -5 gpurun_out/v_${wl}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v_${wl}_$v.json'));print('$wl $v step', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, d['parity'])"
done
done
unset S2C_LIB
echo VAR_DONE
