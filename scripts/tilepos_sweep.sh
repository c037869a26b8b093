# bench C5 at forced tile widths (diagnostic: S2C_TILE_POS overrides the planner)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for tp in ${TPS:-512 256}; do
  S2C_TILE_POS=$tp timeout -k 10 300 python -u bench.py --workload ${WL:-c5} --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tp_$tp.json 2> gpurun_out/tp_$tp.err || { tail -5 gpurun_out/tp_$tp.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/tp_$tp.json'));print($tp, d['ms_per_step'], d['kernels_ms'], d['parity'])"
done
