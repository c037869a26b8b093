# GPU box: C5 whole-vs-streamed CLI with phase times, PMC passes (all four groups for C5,
# C3, C4: instructions, LDS, traffic), the one-wave-per-tile dense variant; each GPU step
# under its own limit, the first failure ends the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-c4}
timeout -k 10 600 python -u scripts/stream_rss.py c5 256 > gpurun_out/stream_rss_c5_$T.json 2> gpurun_out/stream_rss_c5_$T.err || { tail -5 gpurun_out/stream_rss_c5_$T.err; exit 1; }
cat gpurun_out/stream_rss_c5_$T.json; echo
for wl in ${PMC_WLS:-c5 c3 c4}; do
  WL=$wl timeout -k 10 900 bash scripts/pmc.sh || exit 1
done
echo PMC_DONE
S2C_LIB=libs2c_wpt1.so S2C_TILE_POS=512 timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline --no-file-parse > gpurun_out/${T}_c5_wpt1.json 2> gpurun_out/${T}_c5_wpt1.err || { tail -5 gpurun_out/${T}_c5_wpt1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_c5_wpt1.json'));print('c5 wpt1 tp512 step', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, d['parity'])"
echo R03_CALL4_DONE
