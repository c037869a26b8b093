# GPU box, the round's closing evidence in one call: the X-pairs variant of k_tile_dense
# (libs2c_xp.so) through the GPU parity suite; A/B C5 lines against the default build; then
# with the faster build: the default bench line (C5, cpu_baseline legs, file parse), the same
# command under rocprofv3 --kernel-trace --stats, the streamed/whole CLI, the C5 PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-fin}
S2C_LIB=libs2c_xp.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_${T}_xp.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_${T}_xp.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu_${T}_xp.log | head -30; exit $rc; }
for k in 1 2; do
  for lib in libs2c_xp.so libs2c.so; do
    S2C_LIB=$lib timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --no-file-parse \
      > gpurun_out/${T}_ab_${lib}_$k.json 2> gpurun_out/${T}_ab_${lib}_$k.err || { tail -5 gpurun_out/${T}_ab_${lib}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${T}_ab_${lib}_$k.json'));print('$lib', $k, round(d['ms_per_step'],4), round(d['kernels_ms']['step_gpu'],4), round(d['roofline']['frac'],3), d['parity'])"
  done
done
best=$(python - <<PY
import json
def ms(lib):
    return min(json.load(open("gpurun_out/${T}_ab_%s_%d.json" % (lib, k)))["ms_per_step"] for k in (1, 2))
print("libs2c_xp.so" if ms("libs2c_xp.so") < ms("libs2c.so") else "libs2c.so")
PY
) || exit 1
echo "BEST $best"; echo "$best" > gpurun_out/${T}_best.txt
export S2C_LIB=$best
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -5 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_default -o out -- python3 bench.py \
  > gpurun_out/prof_${T}_default.log 2>&1 || { tail -5 gpurun_out/prof_${T}_default.log; exit 1; }
timeout -k 10 600 python -u scripts/stream_rss.py c5 256 > gpurun_out/stream_rss_c5_$T.json 2> gpurun_out/stream_rss_c5_$T.err || { tail -5 gpurun_out/stream_rss_c5_$T.err; exit 1; }
cat gpurun_out/stream_rss_c5_$T.json; echo
WL=c5 timeout -k 10 900 bash scripts/pmc.sh || exit 1
echo R03_FINAL_DONE
