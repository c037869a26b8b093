# round 4: k_tile with half-size layer chunks at 4 waves / SIMD (libs2c_half.so, timing + parity
# of the bench line) against the default build, C4 and C3; the streamed C5 CLI with 64 MB blocks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
WL=c4 TAG=abh4 LIBS="libs2c.so libs2c_half.so" bash scripts/ab_libs.sh || exit 1
S2C_ITEM_SLOTS=1024 WL=c4 TAG=abh4s LIBS="libs2c_half.so" bash scripts/ab_libs.sh || exit 1
WL=c3 TAG=abh3 LIBS="libs2c.so libs2c_half.so" bash scripts/ab_libs.sh || exit 1
timeout -k 10 500 python -u scripts/stream_rss.py c5 256 > gpurun_out/r4h_stream_rss_c5.json 2> gpurun_out/r4h_stream_rss_c5.err || { tail -5 gpurun_out/r4h_stream_rss_c5.err; exit 1; }
tail -2 gpurun_out/r4h_stream_rss_c5.err
