# Round evidence on the GPU box: parity tests, C5 bench line, rocprofv3 kernel stats, PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r02}
STEPS=gpu,bench,prof WLS=${WLS:-c5} TAG=$TAG bash scripts/gpu_check.sh || exit $?
WL=c5 timeout -k 10 900 bash scripts/pmc.sh || exit $?
python scripts/traffic.py c5 $TAG || exit $?
if [ -n "$PMC_C3" ]; then
  WL=c3 TRAFFIC_ONLY=1 timeout -k 10 600 bash scripts/pmc.sh || exit $?
  python scripts/traffic.py c3 $TAG || exit $?
fi
echo ROUND_CHECK_DONE
