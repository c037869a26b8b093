#!/bin/bash
# Ablation sweep of k_pileup over forced tile widths (diagnostic).  TILES="256 512".
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
mkdir -p gpurun_out
for t in ${TILES:-256 512}; do
  echo "tile $t"
  S2C_TILE_POS=$t timeout -k 10 120 python scripts/ablate.py ${WL:-c2} 10 || exit 1
done 2>&1 | grep -v amdgpu.ids
