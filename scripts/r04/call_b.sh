# round 4: timing-only k_tile variants on C4 / C3 (no N-plane pass, no coverage updates), the
# fixed diagnostic build's phase clocks, the C5 8-way shard rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
NOTEST= bash scripts/gpu_iter.sh || exit 1
WL=c4 TAG=abc4 LIBS="libs2c.so libs2c_ablx.so libs2c_abldv.so" bash scripts/ab_libs.sh || exit 1
WL=c3 TAG=abc3 LIBS="libs2c.so libs2c_ablx.so" bash scripts/ab_libs.sh || exit 1
S2C_LIB=libs2c_prof.so timeout -k 10 300 python -u scripts/prof_tile.py c4 0 > gpurun_out/prof_tile_c4.txt 2>&1 || { tail -5 gpurun_out/prof_tile_c4.txt; exit 1; }
cat gpurun_out/prof_tile_c4.txt
timeout -k 10 400 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --no-file-parse --rehearse-shards 8 \
  > gpurun_out/r4_c5_rehearse8.json 2> gpurun_out/r4_c5_rehearse8.err || { tail -5 gpurun_out/r4_c5_rehearse8.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4_c5_rehearse8.json'));s=d['shard_rehearsal'];print('rehearse', d['ms_per_step'], s['projected_ms_per_step'], s['gather_ms'], s['dup_frac'], s['exchange_volumes'])"
