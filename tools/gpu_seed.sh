#!/bin/bash
# seeded-row GPU tests, then bench lines
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_seed_gpu.py} -x -v --timeout 240 --timeout-method thread > gpurun_out/seed_tests.log 2>&1 \
  || { echo SEED TESTS FAILED; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/seed_tests.log | tail -30; exit 1; }
grep -cE "PASSED" gpurun_out/seed_tests.log
BENCH_ARGS="${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu-baseline}" TAG=${TAG:-seed} tools/gpu_bench.sh ${CFGS:-c4 c3}
