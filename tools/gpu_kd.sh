set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kd_tests.log 2>&1 || { echo KD TESTS FAILED; tail -40 gpurun_out/kd_tests.log; exit 1; }
tail -2 gpurun_out/kd_tests.log
timeout -k 10 120 python -u tools/stamps.py --config c4 --sources 512 > gpurun_out/stamps_c4.txt 2>&1; grep -v amdgpu.ids gpurun_out/stamps_c4.txt | tail -24
timeout -k 10 240 python -u bench.py --config c4 --steps 2 --warmup 1 --sources 4096 --no-cpu-baseline --verify 2 > gpurun_out/bench_c4_kd.json 2>gpurun_out/bench_c4_kd.err || { tail gpurun_out/bench_c4_kd.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c4_kd.json'));print('C4 kernel_ms',d['kernel_ms'],'frac',d['roofline']['frac'],d['verified_rows_vs_oracle'])"
timeout -k 10 240 python -u bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --verify 2 > gpurun_out/bench_c3_kd.json 2>gpurun_out/bench_c3_kd.err || { tail gpurun_out/bench_c3_kd.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c3_kd.json'));print('C3 kernel_ms',d['kernel_ms'],'frac',d['roofline']['frac'],d['verified_rows_vs_oracle'])"
