#!/bin/bash
# KD change check: the KD/seed/parity GPU tests, then C4 and C3 bench lines.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
tag=${TAG:-kd}
timeout -k 10 600 python -u -m pytest tests/test_seed_gpu.py tests/test_kd_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/kdcheck_$tag.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error|assert" gpurun_out/kdcheck_$tag.log | head -30; exit 1; }
tail -1 gpurun_out/kdcheck_$tag.log
for cfg in c4 c3; do
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/kdbench_${tag}_$cfg.json 2> gpurun_out/kdbench_${tag}_$cfg.err || { echo BENCH $cfg FAILED; tail -5 gpurun_out/kdbench_${tag}_$cfg.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/kdbench_${tag}_$cfg.json'));print('$cfg', round(d['value']), 'ms', round(d['ms_per_step'],3), d['verified_rows_vs_oracle'])"
done
