# round 4 closing, part 1: PMC passes (instruction mix, LDS, FETCH_SIZE, WRITE_SIZE) of C5 / C4 /
# C3 for traffic.py / bound.py, and C4's work-item size sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
( while true; do date > gpurun_out/heartbeat.txt; sleep 20; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for il in 64 48 40; do
  S2C_ITEM_LAYERS=$il timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --no-file-parse \
    > gpurun_out/g1_c4_il$il.json 2> gpurun_out/g1_c4_il$il.err || { tail -5 gpurun_out/g1_c4_il$il.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/g1_c4_il$il.json'));print('c4 items<=$il', round(d['ms_per_step'],4), d['parity'])"
done
S2C_ITEM_SLOTS=0 timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --no-file-parse \
  > gpurun_out/g1_c4_noshape.json 2> gpurun_out/g1_c4_noshape.err || { tail -5 gpurun_out/g1_c4_noshape.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/g1_c4_noshape.json'));print('c4 no shaping', round(d['ms_per_step'],4), d['parity'])"
for wl in c5 c4 c3; do WL=$wl bash scripts/pmc.sh || exit 1; done
echo G1_DONE
