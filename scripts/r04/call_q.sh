# round 4: k_tile_dense with raised wave priority until a starting wave has issued its window
# loads (s_setprio 3 → 0) against the same build without it, C5, four alternating rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
WL=c5 TAG=abprio1 LIBS="libs2c_noprio.so libs2c_prio.so" bash scripts/ab_libs.sh || exit 1
WL=c5 TAG=abprio2 LIBS="libs2c_prio.so libs2c_noprio.so" bash scripts/ab_libs.sh || exit 1
