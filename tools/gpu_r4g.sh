# round 4: KFH with key filter -- tests, C4f / C3f lines, stamps
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kf_gpu.py > gpurun_out/r4g_tests.log 2>&1 || { tail -30 gpurun_out/r4g_tests.log; exit 1; }
tail -2 gpurun_out/r4g_tests.log
timeout -k 10 600 python -u bench.py --config c4f --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4g_c4f.json 2> gpurun_out/r4g_c4f.err || { tail gpurun_out/r4g_c4f.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4g_c4f.json')); print('c4f', d['ms_per_step'], d['kernel_ms'], d.get('verified_rows_vs_oracle'))"
SHD_ROUTE_KFH=1 timeout -k 10 300 python -u bench.py --config c3f --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4g_c3fh.json 2> gpurun_out/r4g_c3fh.err || { tail gpurun_out/r4g_c3fh.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4g_c3fh.json')); print('c3f KFH', d['ms_per_step'], d.get('verified_rows_vs_oracle'))"
timeout -k 10 300 python -u tools/kf_stamps.py --config c4f --sources 1024 > gpurun_out/kfh_stamps_c4f.txt 2>&1 && cat gpurun_out/kfh_stamps_c4f.txt
