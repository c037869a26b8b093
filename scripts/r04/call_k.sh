# round 4: the whole GPU suite and smoke on the current build, the default C5 bench line, the
# streamed / whole C5 CLI after the host parse changes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4k_smoke.log 2>&1 || { tail -20 gpurun_out/r4k_smoke.log; exit 1; }
tail -2 gpurun_out/r4k_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4k_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4k_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4k_pytest_gpu.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4k_c5_bench.json 2> gpurun_out/r4k_c5_bench.err || { tail -20 gpurun_out/r4k_c5_bench.err; exit 1; }
timeout -k 10 400 python -u scripts/stream_rss.py c5 256 > gpurun_out/r4k_stream_rss_c5.json 2> gpurun_out/r4k_stream_rss_c5.err || { tail -5 gpurun_out/r4k_stream_rss_c5.err; exit 1; }
echo done
