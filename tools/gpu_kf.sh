set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kf_gpu.py tests/test_gpu_parity.py -m gpu -x -v -k "${TESTK:-test}" --timeout 300 --timeout-method thread > gpurun_out/kf_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" gpurun_out/kf_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/kf_tests.log
CFGS="c2f c3f" STEPS=5 bash tools/gpu_abfull.sh "" && CFGS="c2f c3f" STEPS=2 bash tools/gpu_abfull.sh "SHD_ROUTE_KERNEL=f64"
