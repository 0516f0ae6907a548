# round 4: KFH tests + C4f line, first-touch chunk pinning fill
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kf_gpu.py tests/test_topology_gpu.py > gpurun_out/r4f_tests.log 2>&1 || { tail -30 gpurun_out/r4f_tests.log; exit 1; }
tail -2 gpurun_out/r4f_tests.log
timeout -k 10 300 python -u tools/fill_bench.py --configs c3,c4 --out gpurun_out/r4_fill.json > gpurun_out/r4_fill.log 2>&1 || { tail -20 gpurun_out/r4_fill.log; exit 1; }
python -c "import json; [print(r['config'], r['fill_s'], r['triangle_bytes'], r['host_write_GBps'], r.get('engine')) for r in json.load(open('gpurun_out/r4_fill.json'))]"
timeout -k 10 600 python -u bench.py --config c4f --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4f_c4f.json 2> gpurun_out/r4f_c4f.err || { tail gpurun_out/r4f_c4f.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4f_c4f.json')); print('c4f', d['ms_per_step'], d['kernel_ms'], d.get('verified_rows_vs_oracle'), d.get('kernel'))"
timeout -k 10 300 python -u bench.py --config c3f --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4f_c3f.json 2> gpurun_out/r4f_c3f.err || { tail gpurun_out/r4f_c3f.err; exit 1; }
SHD_ROUTE_KFH=1 timeout -k 10 300 python -u bench.py --config c3f --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4f_c3fh.json 2> gpurun_out/r4f_c3fh.err || { tail gpurun_out/r4f_c3fh.err; exit 1; }
python -c "import json; [print(f, json.load(open('gpurun_out/'+f))['ms_per_step']) for f in ('r4f_c3f.json','r4f_c3fh.json')]"
