# round 4: host parse after the single-pass line scanner and the parallel plain-file reads:
# parse_time on the box's 16 threads, then the whole / streamed C5 CLI
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/parse_time.py c5 'S2C_PARSE_THREADS=8' > gpurun_out/r4p_parse_time_c5.json 2> gpurun_out/r4p_parse_time_c5.err || { tail -5 gpurun_out/r4p_parse_time_c5.err; exit 1; }
cat gpurun_out/r4p_parse_time_c5.json
timeout -k 10 400 python -u scripts/stream_rss.py c5 256 > gpurun_out/r4p_stream_rss_c5.json 2> gpurun_out/r4p_stream_rss_c5.err || { tail -5 gpurun_out/r4p_stream_rss_c5.err; exit 1; }
echo done
