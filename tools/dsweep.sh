set -o pipefail
export PYTHONUNBUFFERED=1
for d in 10 15 24 32 48; do
  SHD_ROUTE_DELTA=$d timeout -k 10 120 python -u bench.py --config c4 --steps 2 --warmup 1 --sources 4096 --no-cpu-baseline --verify 1 > gpurun_out/bd.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bd.json'));print('delta $d C4 kernel_ms',round(d['kernel_ms'],2),d['verified_rows_vs_oracle'])"
done
