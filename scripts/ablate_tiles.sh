#!/bin/bash
# Ablation sweep of k_pileup over forced tile widths (diagnostic).  TILES="default 256 512".
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
mkdir -p gpurun_out
for t in ${TILES:-default}; do
  echo "tile $t"
  if [ "$t" = default ]; then
    timeout -k 10 120 python scripts/ablate.py ${WL:-c2} 10 || exit 1
  else
    S2C_TILE_POS=$t timeout -k 10 120 python scripts/ablate.py ${WL:-c2} 10 || exit 1
  fi
done 2>&1 | grep -v amdgpu.ids
