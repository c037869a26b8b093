# bench a workload at forced tile widths (diagnostic: S2C_TILE_POS overrides the planner)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
for wl in ${WLS:-c3}; do
for tp in ${TPS:-512 256}; do
  S2C_TILE_POS=$tp timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-file-parse > gpurun_out/tp_${wl}_$tp.json 2> gpurun_out/tp_${wl}_$tp.err || { tail -5 gpurun_out/tp_${wl}_$tp.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/tp_${wl}_$tp.json'));print('$wl', $tp, round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, d['parity'])"
done
done
