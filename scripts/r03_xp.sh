# GPU box: the X-pairs variant of k_tile_dense (libs2c_xp.so, -DS2C_XPAIRS) through the GPU
# parity suite, then A/B C5 bench lines against the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-xp}
S2C_LIB=libs2c_xp.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_$T.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu_$T.log | head -30; exit $rc; }
for k in 1 2; do
  for lib in libs2c_xp.so libs2c.so; do
    S2C_LIB=$lib timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --no-file-parse \
      > gpurun_out/${T}_${lib}_$k.json 2> gpurun_out/${T}_${lib}_$k.err || { tail -5 gpurun_out/${T}_${lib}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${T}_${lib}_$k.json'));print('$lib', $k, round(d['ms_per_step'],4), round(d['kernels_ms']['step_gpu'],4), round(d['roofline']['frac'],3), d['parity'])"
  done
done
echo R03_XP_DONE
