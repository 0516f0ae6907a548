#!/bin/bash
# One bench line per config given (default: the C4 headline), JSON under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
tag=${TAG:-now}
for cfg in "${@:-c4}"; do
  timeout -k 10 ${BENCH_TIMEOUT:-420} python -u bench.py --config $cfg ${BENCH_ARGS} > gpurun_out/bench_${tag}_$cfg.json 2> gpurun_out/bench_${tag}_$cfg.err \
    || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_${tag}_$cfg.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/bench_${tag}_$cfg.json'));r=d['roofline'];print('$cfg value',round(d['value']),'ms/step',round(d['ms_per_step'],3),'kernel_ms',round(d['kernel_ms'],3),'frac',round(r['frac'],4),'verified',d['verified_rows_vs_oracle'],'cpu',(d.get('cpu_baseline') or {}).get('value'))"
done
