# GPU box: streamed-path GPU tests, whole-vs-streamed CLI wall time on C5 (stream_rss.py), then
# the tile width sweep; each GPU step under its own limit, the first failure ends the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or unsorted or cli" > gpurun_out/pytest_stream.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_stream.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_stream.log | head -30; exit $rc; }
timeout -k 10 600 python -u scripts/stream_rss.py c5 256 > gpurun_out/stream_rss_c5.json 2> gpurun_out/stream_rss_c5.err || { tail -5 gpurun_out/stream_rss_c5.err; exit 1; }
cat gpurun_out/stream_rss_c5.json; echo
if [ -n "$SWEEP" ]; then
  WLS="c3" TPS="${TPS3:-256 384 512}" bash scripts/tilepos_sweep.sh || exit 1
  WLS=c4 TPS="${TPS4:-128 512}" bash scripts/tilepos_sweep.sh || exit 1
fi
echo R03_HOST_DONE
