#!/bin/bash
# k_pileup phase timelines under diagnostic ablations (0x200 no insertions, 0x400 no code stores)
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 1
for x in 0 0x200 0x400 0x600 1; do
  echo "### extra ablate $x"
  timeout -k 10 120 python scripts/phases.py ${WL:-c2} $x 2>&1 | grep -v amdgpu.ids || exit 1
done
