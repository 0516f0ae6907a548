# A/B timing of KD variants on C4: each argument is an env assignment list ("" = default),
# e.g.  bash tools/gpu_ab.sh "" "SHD_ROUTE_KDBLOCK=768"
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CFG=${CFG:-c4}
NSRC=${NSRC:-4096}
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 240 python -u bench.py --config $CFG --steps 2 --warmup 1 --sources $NSRC --no-cpu-baseline --verify 2 \
      > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { echo "variant [$v] failed"; tail -5 gpurun_out/ab_$i.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/ab_$i.json'));print('[$v]', 'kernel_ms', round(d['kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), d['verified_rows_vs_oracle'])"
done
