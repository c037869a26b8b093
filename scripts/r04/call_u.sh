# round 4 final check: smoke, the whole GPU suite and the default bench line on the final build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4u_smoke.log 2>&1 || { tail -20 gpurun_out/r4u_smoke.log; exit 1; }
tail -1 gpurun_out/r4u_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4u_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4u_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4u_pytest_gpu.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4u_c5_bench.json 2> gpurun_out/r4u_c5_bench.err || { tail -20 gpurun_out/r4u_c5_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4u_c5_bench.json'));print('c5 default', round(d['ms_per_step'],4), round(d['roofline']['frac'],3), d['parity'], d['host_parse'])"
