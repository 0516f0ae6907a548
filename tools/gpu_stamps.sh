set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u tools/stamps.py --config ${CFG:-c4} --sources ${NSRC:-512} > gpurun_out/stamps.txt 2>&1; grep -v amdgpu.ids gpurun_out/stamps.txt | tail -30
