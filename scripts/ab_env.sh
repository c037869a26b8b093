# A/B of an environment switch on the C5 bench: alternating runs with and without $AB_ENV
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
for mode in on off; do
  if [ $mode = on ]; then export $AB_ENV=${AB_VAL:-1}; else unset $AB_ENV; fi
  timeout -k 10 300 python -u bench.py --workload ${WL:-c5} --steps 30 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/ab_$mode.json 2> gpurun_out/ab_$mode.err || { tail -5 gpurun_out/ab_$mode.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$mode.json'));print('$AB_ENV $mode step', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()})"
done
done
