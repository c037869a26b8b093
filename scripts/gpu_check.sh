#!/bin/bash
# One gpurun call: GPU parity tests, bench line(s), rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-gpu,bench,prof}
WLS=${WLS:-c5}
TAG=${TAG:-r02}
echo "host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo)" | tee "$OUT/host.txt"
if [[ $STEPS == *gpu* ]]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -3; [ $rc -eq 0 ] || { tail -40 "$OUT/pytest_gpu.log"; echo "pytest gpu rc=$rc"; exit $rc; }
fi
for WL in $WLS; do
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python -u bench.py --workload $WL ${BENCH_ARGS} > "$OUT/bench_${TAG}_$WL.json" 2> "$OUT/bench_${TAG}_$WL.err"
  rc=$?; cat "$OUT/bench_${TAG}_$WL.json"; tail -3 "$OUT/bench_${TAG}_$WL.err"; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
fi
if [[ $STEPS == *prof* ]]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_$WL" -o run \
      -- python3 "$ROOT/bench.py" --workload $WL --steps 10 --warmup 2 --no-cpu-baseline --no-parity \
      > "$OUT/prof_${TAG}_$WL.log" 2>&1
  rc=$?; tail -2 "$OUT/prof_${TAG}_$WL.log"; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; exit $rc; }
  find "$OUT/prof_${TAG}_$WL" -name "*kernel_stats.csv" -exec cat {} \;
  cd "$ROOT"
fi
done
echo ALL_DONE
