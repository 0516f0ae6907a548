# KB fused-path check: KB parity tests, then the C2 bench fused vs unfused.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kb_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/kb_tests.log 2>&1 || { echo KB TESTS FAILED; tail -40 gpurun_out/kb_tests.log; exit 1; }
tail -2 gpurun_out/kb_tests.log
for v in "SHD_ROUTE_KBFUSE=1" "SHD_ROUTE_KBFUSE=0"; do
  env $v timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/kb_$v.json 2> gpurun_out/kb_$v.err || { echo "bench [$v] failed"; tail -5 gpurun_out/kb_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/kb_$v.json'));print('[$v]', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'kernel_ms', round(d['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4), d['verified_rows_vs_oracle'])"
done
CFG=c2 NSRC=2000 timeout -k 10 120 python -u tools/stamps.py --config c2 > gpurun_out/stamps_c2.txt 2>&1; grep -v amdgpu.ids gpurun_out/stamps_c2.txt | tail -8
