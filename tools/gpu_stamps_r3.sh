# stamps of the diagnostic build (per-phase cycles per row) for C4 and C3 planned launches
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/stamps.py --config c4 --plan > gpurun_out/stamps_c4.txt 2>&1 || { tail gpurun_out/stamps_c4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_c4.txt | tail -34
if [ "${C3:-0}" = 1 ]; then
timeout -k 10 200 python -u tools/stamps.py --config c3 --plan > gpurun_out/stamps_c3.txt 2>&1 || { tail gpurun_out/stamps_c3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_c3.txt | tail -34
fi
