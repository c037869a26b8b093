# VALU / LDS / SALU instructions of k_tile_dense per ablation setting (diagnostic build)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
S2C_LIB=libs2c_prof.so timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_abl -o run -- python3 $GRAFT_REPO_ROOT/scripts/prof_dense.py ${WL:-c5} 0,4,2,8,14 > $GRAFT_REPO_ROOT/gpurun_out/pmc_abl.log 2>&1
rc=$?; tail -30 $GRAFT_REPO_ROOT/gpurun_out/pmc_abl.log; exit $rc
