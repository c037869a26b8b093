# round 4: the CLI under option sets the goldens do not use vs the C restatement (reduced
# C5 / C4 / C2 files): same FASTA bytes or the same error
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "options_match" > gpurun_out/r4x_options.log 2>&1 || { tail -40 gpurun_out/r4x_options.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r4x_options.log | tail -10
