# GPU box: A/B C5 bench lines of variant builds (LIBS="libs2c.so libs2c_cp1.so ..."), two rounds,
# each line with its byte-identical parity check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-ab}
for k in 1 2; do
  for lib in ${LIBS:-libs2c.so}; do
    S2C_LIB=$lib timeout -k 10 300 python -u bench.py --workload ${WL:-c5} --steps 20 --warmup 3 --no-cpu-baseline --no-file-parse \
      > gpurun_out/${T}_${lib}_$k.json 2> gpurun_out/${T}_${lib}_$k.err || { tail -5 gpurun_out/${T}_${lib}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${T}_${lib}_$k.json'));print('$lib', $k, round(d['ms_per_step'],4), round(d['kernels_ms']['step_gpu'],4), round(d['roofline']['frac'],3), d['parity'])"
  done
done
echo AB_DONE
