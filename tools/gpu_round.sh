#!/bin/bash
# One GPU call: parity tests, smoke, benches (C2 default, C3, C4 sample).  Stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 120 python -u __graft_entry__.py smoke || exit 1
timeout -k 10 180 python -u bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo BENCH C2 FAILED; tail gpurun_out/bench_c2.err; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 180 python -u bench.py --config c3 --steps 5 --warmup 2 --cpu-budget 5 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { echo BENCH C3 FAILED; tail gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
timeout -k 10 240 python -u bench.py --config c4 --steps 2 --warmup 1 --sources 4096 --cpu-budget 5 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo BENCH C4 FAILED; tail gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
