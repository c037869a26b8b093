# round 4 closing (final build, after the walk-barrier change): C5 PMC passes (traffic / bound), the default bench line and
# its rocprofv3 kernel statistics, C4 / C3 / C2 lines with theirs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
( while true; do date > gpurun_out/heartbeat.txt; sleep 20; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
WL=c5 bash scripts/pmc.sh || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/fin3_c5_default_bench.json 2> gpurun_out/fin3_c5_default_bench.err || { tail -5 gpurun_out/fin3_c5_default_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/fin3_c5_default_bench.json'));print('c5 default', round(d['ms_per_step'],4), round(d['roofline']['frac'],3), d['parity'], d['host_parse_s'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fin3_c5 -o out -- python3 bench.py \
  > gpurun_out/fin3_c5_default_prof.log 2>&1 || { tail -5 gpurun_out/fin3_c5_default_prof.log; exit 1; }
PROF=1 TAG=fin3 WLS="c4 c3 c2" bash scripts/bench_all.sh || exit 1
