#!/bin/bash
# One GPU call: every GPU test, smoke, the driver's default bench line (C4), C3 and C2.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
tag=${TAG:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$tag.log | tail -30; exit 1; }
tail -2 gpurun_out/gpu_tests_$tag.log
timeout -k 10 180 python -u __graft_entry__.py smoke || exit 1
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_${tag}_c4.json 2> gpurun_out/bench_${tag}_c4.err || { echo BENCH C4 FAILED; tail gpurun_out/bench_${tag}_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${tag}_c4.json'));print('C4', round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), d['verified_rows_vs_oracle'], 'cpu', round(d['cpu_baseline']['value'],1))"
for cfg in c3 c2; do
timeout -k 10 240 python -u bench.py --config $cfg --steps 20 --warmup 5 --cpu-budget 5 > gpurun_out/bench_${tag}_$cfg.json 2> gpurun_out/bench_${tag}_$cfg.err || { echo BENCH $cfg FAILED; tail gpurun_out/bench_${tag}_$cfg.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${tag}_$cfg.json'));print('$cfg', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), d['verified_rows_vs_oracle'])"
done
