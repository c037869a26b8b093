# GPU box: deep-path plan sweeps (tile width S2C_TILE_POS, work-item layers S2C_ITEM_LAYERS);
# each bench under its own limit, the first failure ends the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
one() {   # name, workload, env...
  local nm=$1 wl=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-file-parse > gpurun_out/sw_$nm.json 2> gpurun_out/sw_$nm.err || { tail -5 gpurun_out/sw_$nm.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw_$nm.json'));print('$nm', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, d['parity'])"
}
for tp in ${TPS3:-256 320 512}; do one c3_tp$tp c3 S2C_TILE_POS=$tp || exit 1; done
for il in ${ILS4:-32 64 128}; do one c4_il$il c4 S2C_ITEM_LAYERS=$il || exit 1; done
for tp in ${TPS4:-512}; do one c4_tp$tp c4 S2C_TILE_POS=$tp || exit 1; done
echo R03_SWEEP_DONE
