# round 4 closing, part 2: the default bench line (as the driver runs it) and its rocprofv3
# kernel statistics; C4 / C3 / C2 lines with theirs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
( while true; do date > gpurun_out/heartbeat.txt; sleep 20; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u bench.py > gpurun_out/fin_c5_default_bench.json 2> gpurun_out/fin_c5_default_bench.err || { tail -5 gpurun_out/fin_c5_default_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/fin_c5_default_bench.json'));print('c5 default', round(d['ms_per_step'],4), round(d['roofline']['frac'],3), d['parity'], d['cpu_baseline']['value'], d.get('cpu_baseline_mc',{}).get('value'))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fin_c5 -o out -- python3 bench.py \
  > gpurun_out/fin_c5_default_prof.log 2>&1 || { tail -5 gpurun_out/fin_c5_default_prof.log; exit 1; }
PROF=1 TAG=fin WLS="c4 c3 c2" bash scripts/bench_all.sh || exit 1
