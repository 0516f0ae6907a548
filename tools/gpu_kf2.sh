#!/bin/bash
# KF: tests, then fractional benches across bucket widths, then stamps
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kf_gpu.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTK:-kf or kernel_selection}" > gpurun_out/kf_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" gpurun_out/kf_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/kf_tests.log
CFGS="c3f c2f" STEPS=3 bash tools/gpu_abfull.sh "" ${KFVARIANTS} || exit 1
timeout -k 10 200 python -u tools/kf_stamps.py --config c3f ${KFSTAMPENV} > gpurun_out/kf_st.txt 2>&1; timeout -k 10 200 python -u tools/kf_stamps.py --config c2f >> gpurun_out/kf_st.txt 2>&1; grep -v amdgpu.ids gpurun_out/kf_st.txt
