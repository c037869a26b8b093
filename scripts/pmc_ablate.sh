#!/bin/bash
# SQ instruction-mix counters of k_pileup per diagnostic variant (MASKS="0 0x200 ...").
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
WL=${WL:-c2}
GRP=${GRP:-"SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH"}
for m in ${MASKS:-0}; do
  timeout -k 10 120 rocprofv3 --pmc $GRP --output-format csv -d "$OUT/pmca_$WL/m$m" -o run \
      -- python3 "$ROOT/scripts/pmc_run.py" $WL $m > "$OUT/pmca_${WL}_m$m.log" 2>&1 \
      || { echo "pmc mask $m failed"; tail -5 "$OUT/pmca_${WL}_m$m.log"; exit 1; }
done
echo PMC_DONE
