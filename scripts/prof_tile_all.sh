# k_tile phase clocks (diagnostic build libs2c_prof.so) for each workload in $WLS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
for wl in ${WLS:-c3 c4 c2}; do
  S2C_LIB=libs2c_prof.so timeout -k 10 300 python -u scripts/prof_tile.py $wl > gpurun_out/prof_tile_$wl.txt 2>&1 || { tail -5 gpurun_out/prof_tile_$wl.txt; exit 1; }
  echo "== $wl"; cat gpurun_out/prof_tile_$wl.txt
done
