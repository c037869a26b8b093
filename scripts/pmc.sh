#!/bin/bash
# PMC counter passes for the bench workload (one rocprofv3 run per counter group).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
WL=${WL:-c2}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_GROUPS}; do
  i=$((i+1))
  if [ -n "$TRAFFIC_ONLY" ] && [ $i -le 2 ]; then continue; fi   # (FETCH_SIZE / WRITE_SIZE passes only)
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_$WL/p$i" -o run \
      -- python3 "$ROOT/bench.py" --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-file-parse \
      > "$OUT/pmc_${WL}_p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/pmc_${WL}_p$i.log"; exit 1; }
done
echo PMC_DONE
