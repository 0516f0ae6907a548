# KF: one barrier per round again (overflow flag by round parity)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kf_gpu.py > gpurun_out/r4h_tests.log 2>&1 || { tail -30 gpurun_out/r4h_tests.log; exit 1; }
tail -2 gpurun_out/r4h_tests.log
for cfg in c2f c3f; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r4h_$cfg.json 2> gpurun_out/r4h_$cfg.err || { tail gpurun_out/r4h_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4h_$cfg.json')); print('$cfg', d['ms_per_step'], d.get('verified_rows_vs_oracle'))"
done
git_rev=none
