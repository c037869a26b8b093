# round 4: GPU tests, then C4 / C3 / C5 bench lines (k_tile grid shaping), the streamed C5 CLI
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
( while true; do date > gpurun_out/heartbeat.txt; sleep 20; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash scripts/gpu_iter.sh || exit 1
TAG=r4d WLS="c4 c3 c2" bash scripts/bench_all.sh || exit 1
timeout -k 10 500 python -u scripts/stream_rss.py c5 256 > gpurun_out/r4d_stream_rss_c5.json 2> gpurun_out/r4d_stream_rss_c5.err || { tail -5 gpurun_out/r4d_stream_rss_c5.err; exit 1; }
tail -2 gpurun_out/r4d_stream_rss_c5.err
