#!/bin/bash
# The round's GPU steps on the committed tree, one per PART (each GPU step under its own time
# limit; the script stops at the first failure):
#   PART=tests  the whole GPU suite + smoke            -> gpurun_out/<TAG>_gpu_tests.log
#   PART=bench  the bench line of every config (C4, C5 and the fractional configs with their
#               CPU baselines)                         -> gpurun_out/<TAG>_bench_<cfg>.json
#   PART=emul   every rank of a W-way split of C3 and C4 in turn on this GPU (W = 1 2 4 8),
#               plan debug on                          -> gpurun_out/<TAG>_emul_<cfg>.log
#   PART=prof   rocprof kernel stats + PMC passes (tools/prof_round.sh <TAG>)
#   PART=stamps per-phase cycles, diagnostic build (C4 1-GPU and 8-way rank 0, C3)
# usage: TAG=r05 PART=bench bash tools/gpu_round.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05}
case "${PART:-tests}" in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 \
    || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" gpurun_out/${TAG}_gpu_tests.log | tail -30; exit 1; }
  tail -2 gpurun_out/${TAG}_gpu_tests.log
  timeout -k 10 180 python -u __graft_entry__.py smoke || exit 1
  ;;
bench)
  for cfg in ${CFGS:-c4 c3 c2 c5 c3f c2f c4f}; do
    extra=""; steps=20
    [ $cfg = c4f ] && steps=3
    SHD_ROUTE_PLAN_DEBUG=1 timeout -k 10 500 python -u bench.py --config $cfg --steps $steps --warmup 5 $extra \
        > gpurun_out/${TAG}_bench_$cfg.json 2> gpurun_out/${TAG}_bench_$cfg.err || { echo BENCH $cfg FAILED; tail gpurun_out/${TAG}_bench_$cfg.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$cfg.json'));print('$cfg', round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'kernel', round(d['kernel_ms'],3), 'ttt', d.get('time_to_table_ms'), 'frac', round(d['roofline']['frac'],4), 'verified', d.get('verified_rows_vs_oracle'), 'k4', d.get('k4',{}).get('fw_table_ms'), 'cpu', d.get('cpu_baseline') and (round(d['cpu_baseline']['value'],1), d['cpu_baseline']['cores']))"
  done
  ;;
emul)
  for cfg in ${CFGS:-c3 c4}; do
    SHD_ROUTE_PLAN_DEBUG=1 timeout -k 10 500 python -u tools/emul_ranks.py --config $cfg --world ${W:-1 2 4 8} --reps ${REPS:-3} \
        > gpurun_out/${TAG}_emul_$cfg.log 2>&1 || { echo "EMUL $cfg FAILED"; tail -5 gpurun_out/${TAG}_emul_$cfg.log; exit 1; }
    grep -E "^W=[0-9]+:" gpurun_out/${TAG}_emul_$cfg.log
  done
  ;;
prof)
  PROF_PMC=${PROF_PMC:-1} bash tools/prof_round.sh ${TAG}
  ;;
stamps)
  export SHD_ROUTE_LIB=shadow_amd/libshd_route_diag.so
  timeout -k 10 200 python -u tools/stamps.py --config c4 --plan > gpurun_out/${TAG}_stamps_c4.txt 2>&1 &&
  timeout -k 10 200 python -u tools/stamps.py --config c4 --plan --world 8 --rank 0 > gpurun_out/${TAG}_stamps_c4_w8.txt 2>&1 &&
  timeout -k 10 200 python -u tools/stamps.py --config c3 --plan > gpurun_out/${TAG}_stamps_c3.txt 2>&1 || { echo STAMPS FAILED; exit 1; }
  grep -E "total|A_delta|C_lat" gpurun_out/${TAG}_stamps_c4.txt
  ;;
esac
