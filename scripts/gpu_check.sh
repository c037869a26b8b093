#!/bin/bash
# One gpurun call: GPU parity tests, bench line, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-gpu,bench,prof}
WL=${WL:-c2}
echo "host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo)" | tee "$OUT/host.txt"
if [[ $STEPS == *gpu* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread ${PYTEST_ARGS} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -30 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || { echo "pytest gpu rc=$rc"; exit $rc; }
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py --workload $WL ${BENCH_ARGS} > "$OUT/bench_$WL.json" 2> "$OUT/bench_$WL.err"
  rc=$?; cat "$OUT/bench_$WL.json"; tail -5 "$OUT/bench_$WL.err"; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
fi
if [[ $STEPS == *prof* ]]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$WL" -o run \
      -- python3 "$ROOT/bench.py" --workload $WL --steps 10 --warmup 2 --no-cpu-baseline --no-parity \
      > "$OUT/prof_$WL.log" 2>&1
  rc=$?; tail -3 "$OUT/prof_$WL.log"; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; exit $rc; }
  find "$OUT/prof_$WL" -name "*kernel_stats.csv" -exec cat {} \; | head -20
fi
echo ALL_DONE
