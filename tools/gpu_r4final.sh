# Round-4 final checks on the committed tree.  PART=tests: the whole GPU suite + smoke;
# PART=bench: the bench lines of every config (C4 with the CPU baselines); PART=prof: rocprof
# kernel stats + PMC passes (tools/prof_round.sh r04).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
case "${PART:-tests}" in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_gpu_tests.log 2>&1 \
    || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" gpurun_out/r4_gpu_tests.log | tail -30; exit 1; }
  tail -2 gpurun_out/r4_gpu_tests.log
  timeout -k 10 180 python -u __graft_entry__.py smoke || exit 1
  ;;
bench)
  for cfg in c4 c3 c2 c5 c3f c2f c4f; do
    extra="--no-cpu-baseline"; steps=20
    [ $cfg = c4f ] && steps=3
    [ $cfg = c4 ] && extra=""
    [ $cfg = c5 ] && extra=""
    SHD_ROUTE_PLAN_DEBUG=1 timeout -k 10 400 python -u bench.py --config $cfg --steps $steps --warmup 5 $extra > gpurun_out/r4_bench_$cfg.json 2> gpurun_out/r4_bench_$cfg.err || { echo BENCH $cfg FAILED; tail gpurun_out/r4_bench_$cfg.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/r4_bench_$cfg.json'));print('$cfg', round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'kernel', round(d['kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), 'verified', d.get('verified_rows_vs_oracle'), 'k4', d.get('k4',{}).get('fw_table_ms'), 'cpu', d.get('cpu_baseline') and (round(d['cpu_baseline']['value'],1), d['cpu_baseline']['cores']))"
  done
  ;;
prof)
  PROF_PMC=${PROF_PMC:-1} bash tools/prof_round.sh r04
  ;;
esac
