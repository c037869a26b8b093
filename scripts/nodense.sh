# diagnostic: C5 through k_reads + k_tile only (S2C_NO_DENSE), at several tile widths
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for tp in ${TPS:-2048 1024 512}; do
  S2C_NO_DENSE=1 S2C_TILE_POS=$tp timeout -k 10 300 python -u bench.py --workload ${WL:-c5} --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/nd_$tp.json 2> gpurun_out/nd_$tp.err || { tail -5 gpurun_out/nd_$tp.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/nd_$tp.json'));print('nodense tp', $tp, 'step', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, d['parity'])"
done
