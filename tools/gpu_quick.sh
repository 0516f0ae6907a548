# Quick GPU check: all GPU tests, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 240 python -u bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail gpurun_out/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print('C2 value',round(d['value']),'ms/step',round(d['ms_per_step'],4),'kernel_ms',round(d['kernel_ms'],4),'frac',round(d['roofline']['frac'],4),d['verified_rows_vs_oracle'])"
