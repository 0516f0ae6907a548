#!/bin/bash
# One GPU call: tools/gpu_full.sh (every GPU test, smoke, C4/C3/C2 bench lines), then the C5
# bench and the per-phase stamps of the seeded C4 / C3 plans (diagnostic build).
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
tag=${TAG:-r2}
if [ "${SKIP_FULL:-0}" = 0 ]; then TAG=$tag bash tools/gpu_full.sh || exit 1; fi
timeout -k 10 240 python -u bench.py --config c5 --steps 20 --warmup 5 --cpu-budget 5 > gpurun_out/bench_${tag}_c5.json 2> gpurun_out/bench_${tag}_c5.err || { echo BENCH c5 FAILED; tail gpurun_out/bench_${tag}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${tag}_c5.json'));print('c5', round(d['value']), 'ms/step', round(d['ms_per_step'],4), d.get('k4'))"
for cfg in ${STAMP_CFGS:-c4 c3}; do
timeout -k 10 240 python -u tools/stamps.py --config $cfg --plan > gpurun_out/stamps_${tag}_$cfg.txt 2>&1 || { echo STAMPS $cfg FAILED; tail gpurun_out/stamps_${tag}_$cfg.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_${tag}_$cfg.txt
done
