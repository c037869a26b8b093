# round 4: k_tile_dense phase clocks on C5 (prof build: s_memtime per phase per wave)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
S2C_LIB=libs2c_prof.so timeout -k 10 300 python -u scripts/prof_dense.py c5 0,64 > gpurun_out/r4r_dense_phases_c5.txt 2>&1 || { tail -20 gpurun_out/r4r_dense_phases_c5.txt; exit 1; }
cat gpurun_out/r4r_dense_phases_c5.txt
