# round 4: background-pinned fill, new KD / K4 / C3 seed defaults, first C4f line (generic f64)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_topology_gpu.py tests/test_fw_gpu.py tests/test_seed_gpu.py tests/test_library.py} \
  > gpurun_out/r4d_tests.log 2>&1 || { tail -30 gpurun_out/r4d_tests.log; exit 1; }
tail -2 gpurun_out/r4d_tests.log
timeout -k 10 300 python -u tools/fill_bench.py --configs c3,c4 --out gpurun_out/r4_fill.json > gpurun_out/r4_fill.log 2>&1 || { tail -20 gpurun_out/r4_fill.log; exit 1; }
python -c "import json; [print(r['config'], r['layout'], r['fill_s'], r['triangle_bytes'], r['host_write_GBps'], r.get('engine')) for r in json.load(open('gpurun_out/r4_fill.json'))]"
for cfg in c4 c3 c5; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r4d_$cfg.json 2> gpurun_out/r4d_$cfg.err || { tail gpurun_out/r4d_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4d_$cfg.json')); print('$cfg', d['ms_per_step'], d['kernel_ms'], d.get('verified_rows_vs_oracle'), d.get('k4',{}).get('fw_table_ms'))"
done
timeout -k 10 600 python -u bench.py --config c4f --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r4d_c4f.json 2> gpurun_out/r4d_c4f.err || { tail gpurun_out/r4d_c4f.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4d_c4f.json')); print('c4f', d['ms_per_step'], d['kernel_ms'], d.get('verified_rows_vs_oracle'), d['config'])"
