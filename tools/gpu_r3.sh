#!/bin/bash
# Round-3 GPU call: GPU tests (TESTK = pytest -k filter), smoke, the driver's default bench
# line (C4, plan stage times on stderr), and the C5 line with its CPU baselines.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
tag=${TAG:-r3}
if [ -n "${TESTK}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTK}" > gpurun_out/gpu_tests_$tag.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$tag.log | tail -30; exit 1; }
  tail -2 gpurun_out/gpu_tests_$tag.log
fi
timeout -k 10 180 python -u __graft_entry__.py smoke || exit 1
SHD_ROUTE_PLAN_DEBUG=1 timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_${tag}_c4.json 2> gpurun_out/bench_${tag}_c4.err || { echo BENCH C4 FAILED; tail gpurun_out/bench_${tag}_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${tag}_c4.json'));print('C4', round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'plan_s', round(d['plan']['plan_seconds'],4), d['verified_rows_vs_oracle'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
grep -E "plan|closeness" gpurun_out/bench_${tag}_c4.err | tail -3
if [ "${C5:-1}" = 1 ]; then
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 > gpurun_out/bench_${tag}_c5.json 2> gpurun_out/bench_${tag}_c5.err || { echo BENCH C5 FAILED; tail gpurun_out/bench_${tag}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${tag}_c5.json'));print('C5', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'fw', round(d['k4']['fw_table_ms'],3), 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value'],1), d['cpu_baseline_fw'] and d['cpu_baseline_fw']['sample'])"
fi
if [ "${REHEARSE:-0}" = 1 ]; then
# two ranks sharing this box's GPU over gloo: the strong-split path with the triangle payload
SHD_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config ${RCFG:-c3} --steps 5 --warmup 1 --gather-reps 1 > gpurun_out/bench_${tag}_rehearse.json 2> gpurun_out/bench_${tag}_rehearse.err || { echo REHEARSAL FAILED; tail -20 gpurun_out/bench_${tag}_rehearse.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_${tag}_rehearse.json').read().strip().splitlines()[-1]);print('rehearse', json.dumps(d['split']))"
fi
