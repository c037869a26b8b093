# round 4: tests + C5 bench/PMC, A/B of the split-LDS-read variant (+ its PMC), k_tile phase ablations (C4, C3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
PMC=1 bash scripts/gpu_iter.sh || exit 1
LIBS="libs2c.so libs2c_split.so" bash scripts/ab_libs.sh || exit 1
cd /tmp
S2C_LIB=libs2c_split.so timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_split_c5 -o run \
    -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-file-parse \
    > $GRAFT_REPO_ROOT/gpurun_out/pmc_split.log 2>&1 || { echo "pmc failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc_split.log; exit 1; }
cd $GRAFT_REPO_ROOT
echo "== split variant"; python3 scripts/pmc_summary.py gpurun_out/pmc_split_c5 k_tile | grep -E "VALU|LDS|WAVES|duration"
WL=c4 ABLS="0 1 2 4" bash scripts/pmc_abl_tile.sh > gpurun_out/tabl_c4.txt 2>&1 || { tail -20 gpurun_out/tabl_c4.txt; exit 1; }
cat gpurun_out/tabl_c4.txt
WL=c3 ABLS="0 2" bash scripts/pmc_abl_tile.sh > gpurun_out/tabl_c3.txt 2>&1 || { tail -20 gpurun_out/tabl_c3.txt; exit 1; }
cat gpurun_out/tabl_c3.txt
