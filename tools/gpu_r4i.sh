# device seed forest for multi-rank plans: tests, plan stage times, 8-way emulation
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_seed_gpu.py tests/test_multiproc_gpu.py > gpurun_out/r4i_tests.log 2>&1 || { tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -2 gpurun_out/r4i_tests.log
timeout -k 10 300 python -u tools/plan_debug.py > gpurun_out/plandbg.txt 2>&1 && grep "W=" gpurun_out/plandbg.txt
timeout -k 10 400 python -u tools/emul_ranks.py --config c4 --world 2 8 > gpurun_out/r4_emul.log 2>&1 && tail -3 gpurun_out/r4_emul.log
