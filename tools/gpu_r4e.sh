# round 4: fill with first-touch chunk pinning (tests of the front end + fill bench)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_topology_gpu.py > gpurun_out/r4e_tests.log 2>&1 || { tail -30 gpurun_out/r4e_tests.log; exit 1; }
tail -2 gpurun_out/r4e_tests.log
timeout -k 10 300 python -u tools/fill_bench.py --configs c3,c4 --out gpurun_out/r4_fill.json > gpurun_out/r4_fill.log 2>&1 || { tail -20 gpurun_out/r4_fill.log; exit 1; }
python -c "import json; [print(r['config'], r['fill_s'], r['triangle_bytes'], r['host_write_GBps'], r.get('engine')) for r in json.load(open('gpurun_out/r4_fill.json'))]"
