set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
S2C_LIB=libs2c_prof.so timeout -k 10 300 python -u scripts/prof_tile.py ${WL:-c2} > gpurun_out/prof_tile.txt 2>&1; rc=$?; cat gpurun_out/prof_tile.txt; exit $rc
