# round 4: host memory and wall time of the whole-batch CLI vs streamed batches (stream_rss.py)
# on C5's coordinate-sorted .sam and C3's shuffled BGZF .sam.gz; a heartbeat file while they run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
( while true; do date > gpurun_out/heartbeat.txt; sleep 20; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 500 python -u scripts/stream_rss.py c5 256 > gpurun_out/r4_stream_rss_c5.json 2> gpurun_out/r4_stream_rss_c5.err || { tail -5 gpurun_out/r4_stream_rss_c5.err; exit 1; }
cat gpurun_out/r4_stream_rss_c5.err | tail -3; cat gpurun_out/r4_stream_rss_c5.json
timeout -k 10 800 python -u scripts/stream_rss.py c3 256 > gpurun_out/r4_stream_rss_c3.json 2> gpurun_out/r4_stream_rss_c3.err || { tail -5 gpurun_out/r4_stream_rss_c3.err; exit 1; }
cat gpurun_out/r4_stream_rss_c3.err | tail -3; cat gpurun_out/r4_stream_rss_c3.json
