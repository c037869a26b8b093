# VALU / SALU / LDS instructions and LDS conflicts of k_tile_dense per ablated phase (prof build:
# `make prof`).  One rocprofv3 run per ablation setting so each directory holds one setting.
#   ABLS="0 2 4 8 16 32 62" WL=c5 bash scripts/pmc_abl_dense.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/pmc_abl_${WL:-c5}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for b in ${ABLS:-0 2 4 8 16 32 62}; do
  S2C_LIB=libs2c_prof.so timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$OUT/a$b" -o run \
      -- python3 "$ROOT/scripts/prof_dense.py" ${WL:-c5} $b > "$OUT/a$b.log" 2>&1 || { echo "ablation $b failed"; tail -5 "$OUT/a$b.log"; exit 1; }
  echo "== ablate $b"; python3 "$ROOT/scripts/pmc_summary.py" "$OUT/a$b" k_tile_dense | grep -E "INSTS|WAVES|LDS|duration"
done
