# GPU box: parity suite, C2-C4 bench + kernel stats at the planner's 512-position deep tiles,
# deep-tile / item sweeps, C5 dense ablation clocks; each GPU step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-c3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_$T.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu_$T.log | head -30; exit $rc; }
TAG=$T PROF=1 WLS="c3 c4 c2" bash scripts/bench_all.sh || exit 1
one() {
  local nm=$1 wl=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-file-parse > gpurun_out/sw_$nm.json 2> gpurun_out/sw_$nm.err || { tail -5 gpurun_out/sw_$nm.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw_$nm.json'));print('$nm', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, d['parity'])"
}
one c3_dt1024 c3 S2C_DEEP_TILE=1024 || exit 1
one c4_dt1024 c4 S2C_DEEP_TILE=1024 || exit 1
one c4_il32 c4 S2C_ITEM_LAYERS=32 || exit 1
one c2_dt1024 c2 S2C_DEEP_TILE=1024 || exit 1
timeout -k 10 300 python -u scripts/prof_dense.py c5 0,2,4,8 > gpurun_out/${T}_prof_dense.txt 2>&1 || { tail -5 gpurun_out/${T}_prof_dense.txt; exit 1; }
cat gpurun_out/${T}_prof_dense.txt
echo R03_CALL3_DONE
