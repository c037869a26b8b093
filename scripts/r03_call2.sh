# GPU box: parity suite, C5 bench + kernel stats, deep-path sweeps, C3 PMC (instruction and
# LDS counters), host parse A/B; each GPU step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-c2}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_$T.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert|FAIL" gpurun_out/pytest_gpu_$T.log | head -30; exit $rc; }
TAG=$T PROF=1 WLS="c5" bash scripts/bench_all.sh || exit 1
bash scripts/r03_sweep.sh || exit 1
if [ -n "$PMC" ]; then
  ( cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_${T}_c3/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-file-parse > $GRAFT_REPO_ROOT/gpurun_out/pmc_${T}_c3_p1.log 2>&1 ) || { echo "pmc p1 failed"; exit 1; }
  ( cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_${T}_c3/p2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-file-parse > $GRAFT_REPO_ROOT/gpurun_out/pmc_${T}_c3_p2.log 2>&1 ) || { echo "pmc p2 failed"; exit 1; }
  echo PMC_OK
fi
timeout -k 10 600 python -u scripts/parse_time.py c5 'S2C_HUGEPAGES=0' 'S2C_HUGE_MIN_KB=1024' 'S2C_HOST_TIMING=1' > gpurun_out/parse_time_$T.json 2> gpurun_out/parse_time_$T.err || { tail -5 gpurun_out/parse_time_$T.err; exit 1; }
cat gpurun_out/parse_time_$T.json; echo
echo R03_CALL2_DONE
