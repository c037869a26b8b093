# round 4: the full-size C3 .sam.gz golden through the product parser (now always on)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread --durations=5 -k "config_fasta and c3" > gpurun_out/r4o_c3gz_golden.log 2>&1 || { tail -30 gpurun_out/r4o_c3gz_golden.log; exit 1; }
tail -12 gpurun_out/r4o_c3gz_golden.log
