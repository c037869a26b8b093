# round 4: pipelined streamed snapshots (s2c_parser_detach / _attach) — GPU stream tests, then
# the streamed C5 / C3 CLI against the whole-batch path, pipelined and serial
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "stream" > gpurun_out/r4i_pytest_stream.log 2>&1 || { tail -20 gpurun_out/r4i_pytest_stream.log; exit 1; }
tail -2 gpurun_out/r4i_pytest_stream.log
timeout -k 10 400 python -u scripts/stream_rss.py c5 256 > gpurun_out/r4i_stream_rss_c5.json 2> gpurun_out/r4i_stream_rss_c5.err || { tail -5 gpurun_out/r4i_stream_rss_c5.err; exit 1; }
S2C_STREAM_PIPE=0 timeout -k 10 400 python -u scripts/stream_rss.py c5 256 > gpurun_out/r4i_stream_rss_c5_serial.json 2> gpurun_out/r4i_stream_rss_c5_serial.err || { tail -5 gpurun_out/r4i_stream_rss_c5_serial.err; exit 1; }
timeout -k 10 400 python -u scripts/stream_rss.py c3 256 > gpurun_out/r4i_stream_rss_c3.json 2> gpurun_out/r4i_stream_rss_c3.err || { tail -5 gpurun_out/r4i_stream_rss_c3.err; exit 1; }
echo done
