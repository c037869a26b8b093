set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
S2C_LIB=libs2c_prof.so timeout -k 10 300 python -u scripts/prof_tile.py ${WL:-c2} > gpurun_out/prof_tile.txt 2>&1; rc=$?; cat gpurun_out/prof_tile.txt; [ $rc -eq 0 ] || exit $rc
for wl in ${WLS:-c2}; do
timeout -k 10 300 python -u bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_$wl.json 2> gpurun_out/b_$wl.err || { tail -5 gpurun_out/b_$wl.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_$wl.json'));print('$wl step', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, d['parity'])"
done
