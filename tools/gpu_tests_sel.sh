#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS} -x -v --timeout 300 --timeout-method thread > gpurun_out/sel_tests.log 2>&1 || { echo TESTS FAILED; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/sel_tests.log | tail -40; exit 1; }
grep -cE "PASSED" gpurun_out/sel_tests.log; tail -1 gpurun_out/sel_tests.log
