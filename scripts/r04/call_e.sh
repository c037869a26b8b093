# round 4: k_tile with the piece records / op words issued a layer ahead — GPU tests, A/B
# against the previous kernels on C4 / C3, phase clocks and PMC of C4, the streamed C5 CLI
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
( while true; do date > gpurun_out/heartbeat.txt; sleep 20; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
NOTEST= TPS=0 bash scripts/gpu_iter.sh || exit 1
WL=c4 TAG=abe4 LIBS="libs2c.so libs2c_prev.so" bash scripts/ab_libs.sh || exit 1
WL=c3 TAG=abe3 LIBS="libs2c.so libs2c_prev.so" bash scripts/ab_libs.sh || exit 1
S2C_LIB=libs2c_prof.so timeout -k 10 300 python -u scripts/prof_tile.py c4 0 > gpurun_out/prof_tile_c4e.txt 2>&1 || { tail -5 gpurun_out/prof_tile_c4e.txt; exit 1; }
grep -E "pileup|cyc/wg|layers" gpurun_out/prof_tile_c4e.txt
NOTEST=1 PMC=1 WL=c4 bash scripts/gpu_iter.sh || exit 1
timeout -k 10 500 python -u scripts/stream_rss.py c5 256 > gpurun_out/r4e_stream_rss_c5.json 2> gpurun_out/r4e_stream_rss_c5.err || { tail -5 gpurun_out/r4e_stream_rss_c5.err; exit 1; }
tail -2 gpurun_out/r4e_stream_rss_c5.err
