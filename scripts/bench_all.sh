# Bench every workload in $WLS (device step only: no CPU baselines, no file parse), then, with
# PROF=1, rocprofv3 kernel stats of each; every GPU step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-ba}
for wl in ${WLS:-c5 c3 c4 c2}; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-file-parse \
    > gpurun_out/${TAG}_$wl.json 2> gpurun_out/${TAG}_$wl.err || { tail -5 gpurun_out/${TAG}_$wl.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$wl.json'));print('$wl step', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'frac', round(d['roofline']['frac'],3), d['parity'])"
  if [ -n "$PROF" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$wl -o out -- \
      python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-file-parse --no-parity \
      > gpurun_out/prof_${TAG}_$wl.log 2>&1 || { tail -5 gpurun_out/prof_${TAG}_$wl.log; exit 1; }
  fi
done
echo BENCH_ALL_DONE
