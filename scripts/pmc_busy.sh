# VALU / LDS / SALU busy cycles of the bench kernels (one rocprofv3 --pmc pass)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/avail.txt 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_busy -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload ${WL:-c5} --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/pmc_busy.log 2>&1
rc=$?; tail -3 $GRAFT_REPO_ROOT/gpurun_out/pmc_busy.log; exit $rc
