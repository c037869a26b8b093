# GPU box, one call: GPU parity suite, every workload's bench + rocprof kernel stats, the C5
# whole-vs-streamed CLI, then experiments (C5 at 2048-position tiles, dense phase clocks,
# the 8-way shard rehearsal).  Every GPU step under its own limit; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-rd}
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu_$T.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_gpu_$T.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu_$T.log | head -30; exit $rc; }
fi
TAG=$T PROF=${PROF:-1} WLS="${WLS:-c5 c3 c4 c2}" bash scripts/bench_all.sh || exit 1
if [ -z "$NOHOST" ]; then
  timeout -k 10 600 python -u scripts/stream_rss.py c5 256 > gpurun_out/stream_rss_c5_$T.json 2> gpurun_out/stream_rss_c5_$T.err || { tail -5 gpurun_out/stream_rss_c5_$T.err; exit 1; }
  cat gpurun_out/stream_rss_c5_$T.json; echo
fi
if [ -n "$EXP" ]; then
  timeout -k 10 300 python -u scripts/prof_dense.py c5 ${ABL:-0} > gpurun_out/${T}_prof_dense.txt 2>&1 || { tail -5 gpurun_out/${T}_prof_dense.txt; exit 1; }
  cat gpurun_out/${T}_prof_dense.txt
  timeout -k 10 400 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline --no-file-parse --rehearse-shards 8 > gpurun_out/${T}_c5_shards8.json 2> gpurun_out/${T}_c5_shards8.err || { tail -5 gpurun_out/${T}_c5_shards8.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_c5_shards8.json'));print('c5 shards8', d['shard_rehearsal'])"
fi
echo R03_ROUND_DONE
