#!/bin/bash
# seeded tests, then C4/C3 bench lines under planner options (SHD_ROUTE_SEED_ROOTS / _DEPTH);
# SWEEP entries are cfg:VAR=val+VAR2=val2
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_seed_gpu.py} -x -v --timeout 240 --timeout-method thread > gpurun_out/seed_tests.log 2>&1 \
  || { echo SEED TESTS FAILED; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/seed_tests.log | tail -30; exit 1; }
grep -cE "PASSED" gpurun_out/seed_tests.log
fi
for spec in ${SWEEP:-"c4:" "c3:" "c3:SHD_ROUTE_SEED_ROOTS=1024" "c3:SHD_ROUTE_SEED_DEPTH=6"}; do
  cfg=${spec%%:*}; envs=$(echo "${spec#*:}" | tr "+" " ")
  tag=$(echo "$cfg$envs" | tr -c 'a-zA-Z0-9' '_')
  env $envs timeout -k 10 300 python -u bench.py --config $cfg ${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu-baseline --verify 2} > gpurun_out/sw_$tag.json 2> gpurun_out/sw_$tag.err \
    || { echo "bench $spec failed"; tail -5 gpurun_out/sw_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw_$tag.json'));p=d['plan'];print('$spec','ms/step',round(d['ms_per_step'],3),'frac',round(d['roofline']['frac'],3),'ok',d['verified_rows_vs_oracle'],'roots',p['roots'],'levels',p['levels'],'stored',p['stored_rows'],'plan_s',round(p['plan_seconds'],2))"
done
