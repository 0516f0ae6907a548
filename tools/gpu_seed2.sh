#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
SWEEP="c4:SHD_ROUTE_SEEDS=1 c4:SHD_ROUTE_SEEDS=2 c4:SHD_ROUTE_SEEDS=3 c3:SHD_ROUTE_SEEDS=1 c3:SHD_ROUTE_SEEDS=2 c3:SHD_ROUTE_SEEDS=3" tools/gpu_seed_sweep.sh || exit 1
timeout -k 10 200 python -u tools/stamps.py --config c4 --plan > gpurun_out/stamps_c4_plan2.txt 2>&1 && grep -v amdgpu.ids gpurun_out/stamps_c4_plan2.txt | head -30
