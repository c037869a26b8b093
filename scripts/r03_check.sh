# GPU box: full GPU parity suite, then every workload's bench (device step) and, with HOST=1,
# the whole-vs-streamed C5 CLI (stream_rss.py); every GPU step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
fi
TAG=${TAG:-ck} WLS="${WLS:-c5 c3 c4 c2}" bash scripts/bench_all.sh || exit 1
if [ -n "$HOST" ]; then
  timeout -k 10 600 python -u scripts/stream_rss.py c5 256 > gpurun_out/stream_rss_c5.json 2> gpurun_out/stream_rss_c5.err || { tail -5 gpurun_out/stream_rss_c5.err; exit 1; }
  cat gpurun_out/stream_rss_c5.json; echo
fi
echo R03_CHECK_DONE
