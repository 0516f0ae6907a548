#!/bin/bash
# A/B of full-table benches: TESTK (pytest -k filter, optional) first, then for each config in
# CFGS (default "c4 c3") each variant argument (an env assignment list, "" = default) is run as
# a 5-step bench line; prints ms/step and the rows kernel time.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "${TESTK}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTK}" > gpurun_out/abf_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" gpurun_out/abf_tests.log | tail -30; exit 1; }
  tail -1 gpurun_out/abf_tests.log
fi
i=0
for cfg in ${CFGS:-c4 c3}; do
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --verify 4 \
        > gpurun_out/abf_$i.json 2> gpurun_out/abf_$i.err || { echo "variant [$v] $cfg failed"; tail -5 gpurun_out/abf_$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abf_$i.json'));print('$cfg [$v]', 'ms/step', round(d['ms_per_step'],3), 'kernel_ms', round(d['kernel_ms'],3), 'verified', d['verified_rows_vs_oracle'])"
  done
done
