# round 4: the new/changed GPU tests, then the end-to-end fill bench (C3, C4)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_payload_gpu.py tests/test_kf_gpu.py tests/test_topology_gpu.py \
  "tests/test_seed_gpu.py::test_c3_writer_ring_no_stall" "tests/test_seed_gpu.py::test_c3_eight_rank_plans_every_row" \
  > gpurun_out/r4b_tests.log 2>&1 || { tail -30 gpurun_out/r4b_tests.log; exit 1; }
tail -3 gpurun_out/r4b_tests.log
timeout -k 10 300 python -u tools/fill_bench.py --configs c3,c4 --out gpurun_out/r4_fill.json > gpurun_out/r4_fill.log 2>&1 || { tail -20 gpurun_out/r4_fill.log; exit 1; }
python -c "import json; [print(r['config'], r['layout'], r['fill_s'], r['triangle_bytes'], r['host_write_GBps'], r.get('engine',{}).get('fill_warm_s')) for r in json.load(open('gpurun_out/r4_fill.json'))]"
