# VALU / SALU / LDS instructions and LDS conflicts of k_tile per ablated phase (prof build:
# `make prof`; bits 1 walk, 2 count, 4 flush atomics).  One rocprofv3 run per setting.
#   ABLS="0 1 2 4" WL=c3 bash scripts/pmc_abl_tile.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/pmc_tabl_${WL:-c3}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for b in ${ABLS:-0 1 2 4 3}; do
  S2C_LIB=libs2c_prof.so timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$OUT/a$b" -o run \
      -- python3 "$ROOT/scripts/prof_tile.py" ${WL:-c3} $b > "$OUT/a$b.log" 2>&1 || { echo "ablation $b failed"; tail -5 "$OUT/a$b.log"; exit 1; }
  echo "== ablate $b"; grep -E "pileup|cyc/wg|layers" "$OUT/a$b.log"; python3 "$ROOT/scripts/pmc_summary.py" "$OUT/a$b" "k_tile<" | grep -E "INSTS|WAVES|LDS|duration"
done
