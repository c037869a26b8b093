#!/bin/bash
# One parameterised GPU-box runner (replaces round 4's one-script-per-call files).
#
#   bash scripts/run.sh STEP [STEP ...]      (every step under its own time limit; the first
#                                              failing step ends the run)
# Steps (outputs under gpurun_out/, prefixed with $TAG, default "r"):
#   smoke                 __graft_entry__.smoke()
#   tests                 pytest -m gpu (PYTEST_K: -k expression; default the whole suite)
#   quick                 pytest -m gpu on the dense-path subset
#   bench:WL              bench line of workload WL (device step; no CPU legs)
#   default               the default `python bench.py` (the driver's line, CPU legs included)
#   ab:WL                 A/B of LIBS="libs2c.so libs2c_x.so ..." on WL, two rounds (the second in reverse order)
#   abenv:WL              A/B of libs2c.so without / with the environment ENVB (e.g. "S2C_NO_TILE_EVENTS=1")
#   prof:WL               rocprofv3 --kernel-trace --stats of WL's bench line
#   profdefault           rocprofv3 --kernel-trace --stats of the default bench line
#   pmc:WL                PMC passes of WL (scripts/pmc.sh)
#   phases:WL             phase clocks of the dense kernel (libs2c_prof.so, scripts/prof_dense.py)
#   tphases:WL            phase clocks of k_tile (libs2c_prof.so, scripts/prof_tile.py)
#   valu:WL               VALU per phase of k_tile_dense (prof-build ablations, one PMC pass)
#   poison                pytest -m gpu on the LDS-poison build (libs2c_poison.so)
#   rehearse:N            bench --rehearse-shards N (the one-GPU rehearsal of the N-way split)
#   bench2[:WL]           bench.py --gpus 2 (strong split + weak run), 2 ranks sharing the GPU over gloo
#   streamrss:WL          whole vs streamed CLI on WL's .sam (scripts/stream_rss.py: time, peak RSS, FASTA sha)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r}
( while true; do date > gpurun_out/heartbeat.txt; sleep 20; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
NB="--no-cpu-baseline --no-file-parse"
line() {   # print the headline fields of a bench JSON
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items() if isinstance(v,(int,float))}, 'frac', round(d['roofline']['frac'],3), d['parity'])" "$1" "$2"
}
for st in "$@"; do
  name=${st%%:*}; arg=${st#*:}; [ "$arg" = "$st" ] && arg=""
  echo "== $st"
  case $name in
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 \
        || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
      tail -2 gpurun_out/${T}_smoke.log ;;
    tests|quick)
      K=${PYTEST_K:-}
      [ $name = quick ] && K=${PYTEST_K:-dense or c5 or hip_path or batch_model}
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
        > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
      tail -3 gpurun_out/${T}_pytest_gpu.log
      [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/${T}_pytest_gpu.log | head -30; exit $rc; } ;;
    bench)
      timeout -k 10 300 python -u bench.py --workload $arg --steps ${STEPS:-20} --warmup 3 $NB \
        > gpurun_out/${T}_${arg}_bench.json 2> gpurun_out/${T}_${arg}_bench.err || { tail -5 gpurun_out/${T}_${arg}_bench.err; exit 1; }
      line gpurun_out/${T}_${arg}_bench.json $arg ;;
    default)
      timeout -k 10 600 python -u bench.py > gpurun_out/${T}_default_bench.json 2> gpurun_out/${T}_default_bench.err \
        || { tail -5 gpurun_out/${T}_default_bench.err; exit 1; }
      line gpurun_out/${T}_default_bench.json default ;;
    ab)
      for k in 1 2; do
        L=${LIBS:-libs2c.so}; [ $k = 2 ] && L=$(echo $L | tr ' ' '\n' | tac | tr '\n' ' ')   # (second round in reverse order: the first run of a pair measured ~1-3 % faster)
        for lib in $L; do
          S2C_LIB=$lib timeout -k 10 300 python -u bench.py --workload $arg --steps 20 --warmup 3 $NB \
            > gpurun_out/${T}_${arg}_${lib}_$k.json 2> gpurun_out/${T}_${arg}_${lib}_$k.err || { tail -5 gpurun_out/${T}_${arg}_${lib}_$k.err; exit 1; }
          line gpurun_out/${T}_${arg}_${lib}_$k.json "$arg $lib $k"
        done
      done ;;
    abenv)
      for k in 1 2; do
        VS="base env"; [ $k = 2 ] && VS="env base"
        for v in $VS; do
          E=""; [ $v = env ] && E="$ENVB"
          env $E timeout -k 10 300 python -u bench.py --workload $arg --steps 20 --warmup 3 $NB \
            > gpurun_out/${T}_${arg}_${v}_$k.json 2> gpurun_out/${T}_${arg}_${v}_$k.err || { tail -5 gpurun_out/${T}_${arg}_${v}_$k.err; exit 1; }
          line gpurun_out/${T}_${arg}_${v}_$k.json "$arg $v $k"
        done
      done ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_$arg -o out -- \
        python3 bench.py --workload $arg --steps 10 --warmup 2 $NB --no-parity > gpurun_out/${T}_prof_$arg.log 2>&1 \
        || { tail -5 gpurun_out/${T}_prof_$arg.log; exit 1; } ;;
    profdefault)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_default -o out -- \
        python3 bench.py > gpurun_out/${T}_prof_default.log 2>&1 || { tail -5 gpurun_out/${T}_prof_default.log; exit 1; } ;;
    pmc)
      WL=$arg bash scripts/pmc.sh || exit 1 ;;
    phases)
      S2C_LIB=libs2c_prof.so timeout -k 10 300 python -u scripts/prof_dense.py $arg 0 > gpurun_out/${T}_phases_$arg.txt 2>&1 \
        || { tail -9 gpurun_out/${T}_phases_$arg.txt; exit 1; }
      tail -12 gpurun_out/${T}_phases_$arg.txt ;;
    tphases)
      S2C_LIB=libs2c_prof.so timeout -k 10 300 python -u scripts/prof_tile.py $arg > gpurun_out/${T}_tphases_$arg.txt 2>&1 \
        || { tail -9 gpurun_out/${T}_tphases_$arg.txt; exit 1; }
      tail -12 gpurun_out/${T}_tphases_$arg.txt ;;
    valu)     # VALU per phase of k_tile_dense: prof build ablations under one SQ_INSTS_VALU pass (scripts/valu_phases.py)
      S2C_LIB=libs2c_prof.so timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv \
        -d gpurun_out/${T}_valu_$arg -o run -- python3 scripts/prof_dense.py $arg 0,4,2,8,16,32,64 \
        > gpurun_out/${T}_valu_$arg.log 2>&1 || { tail -9 gpurun_out/${T}_valu_$arg.log; exit 1; }
      python scripts/valu_phases.py gpurun_out/${T}_valu_$arg 0,4,2,8,16,32,64 > gpurun_out/${T}_valu_$arg.txt 2>&1
      cat gpurun_out/${T}_valu_$arg.txt ;;
    poison)   # the GPU suite once on the LDS-poison build (make poison): every kernel's LDS 0xA5 at entry
      S2C_LIB=libs2c_poison.so timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > gpurun_out/${T}_pytest_gpu_poison.log 2>&1; rc=$?
      tail -3 gpurun_out/${T}_pytest_gpu_poison.log
      [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/${T}_pytest_gpu_poison.log | head -30; exit $rc; } ;;
    rehearse)
      timeout -k 10 600 python -u bench.py --rehearse-shards $arg > gpurun_out/${T}_rehearse_$arg.json 2> gpurun_out/${T}_rehearse_$arg.err \
        || { tail -5 gpurun_out/${T}_rehearse_$arg.err; exit 1; } ;;
    bench2)   # bench.py --gpus 2 as the driver runs it (torchrun started as a child), both ranks sharing the GPU over gloo
      S2C_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 3 --workload ${arg:-c5} \
        --no-cpu-baseline > gpurun_out/${T}_bench_2rank.json 2> gpurun_out/${T}_bench_2rank.err \
        || { tail -20 gpurun_out/${T}_bench_2rank.err; exit 1; }
      line gpurun_out/${T}_bench_2rank.json "2rank" ;;
    streamrss)
      timeout -k 10 900 python -u scripts/stream_rss.py $arg > gpurun_out/${T}_stream_rss_$arg.json 2> gpurun_out/${T}_stream_rss_$arg.err \
        || { tail -5 gpurun_out/${T}_stream_rss_$arg.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print({k:(d[k]['seconds'],d[k]['peak_rss_mb']) for k in d if k.startswith('whole') or k.startswith('stream')}, d['identical']);[print(k,d[k]['phases_s']) for k in d if k.startswith('whole')]" gpurun_out/${T}_stream_rss_$arg.json ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo RUN_DONE
