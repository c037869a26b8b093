# round 4: streamed CLI with the SO header check — the streamed GPU tests, then C3 .sam.gz
# whole vs streamed
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "stream or unsorted" > gpurun_out/r4y_stream_tests.log 2>&1 || { tail -40 gpurun_out/r4y_stream_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4y_stream_tests.log | tail -2
timeout -k 10 500 python -u scripts/stream_rss.py c3 256 > gpurun_out/r4y_stream_rss_c3.json 2> gpurun_out/r4y_stream_rss_c3.err || { tail -5 gpurun_out/r4y_stream_rss_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4y_stream_rss_c3.json'));print({m: (d[m]['seconds'], d[m]['peak_rss_mb']) for m in ('whole','stream')}, d['identical'])"
