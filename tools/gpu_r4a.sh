# round 4 first look: production-default stamps (diagnostic build, KD_PREW 0) for C4 and C3, and a C4 bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u tools/stamps.py --config c4 --plan > gpurun_out/r4_stamps_c4.txt 2>&1 || { tail gpurun_out/r4_stamps_c4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_stamps_c4.txt | tail -34
timeout -k 10 200 python -u tools/stamps.py --config c3 --plan > gpurun_out/r4_stamps_c3.txt 2>&1 || { tail gpurun_out/r4_stamps_c3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_stamps_c3.txt | tail -34
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4a_c4.json 2> gpurun_out/r4a_c4.err || { tail gpurun_out/r4a_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4a_c4.json')); print('C4', d['ms_per_step'], d['kernel_ms'], d['plan']['plan_seconds'])"
