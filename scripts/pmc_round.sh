#!/bin/bash
# PMC passes (scripts/pmc.sh) for each workload in $WLS; traffic/bound JSON are derived
# afterwards on the host from gpurun_out/pmc_<wl> (scripts/traffic.py, scripts/bound.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for wl in ${WLS:-c5 c3}; do
  WL=$wl timeout -k 10 900 bash scripts/pmc.sh || exit $?
done
echo PMC_ROUND_DONE
