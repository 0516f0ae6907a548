# A/B of KD knobs on one box: bench (C4 by default, CFG=c3 for C3) once per env setting, kernel
# time + oracle verification per line.  Usage: bash tools/gpu_ab4.sh "A=1" "A=1 B=2" ...
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CFG=${CFG:-c4}
STEPS=${STEPS:-10}
i=0
for setting in "" "$@"; do
  i=$((i+1))
  env $setting timeout -k 10 300 python -u bench.py --config $CFG --steps $STEPS --warmup 2 --no-cpu-baseline --verify 4 \
      > gpurun_out/ab4_$i.json 2> gpurun_out/ab4_$i.err || { echo "FAILED: $setting"; tail -5 gpurun_out/ab4_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab4_$i.json')); print('%-40s step %.3f kernel %.3f plan %.1f verified %s' % (sys.argv[1] or 'baseline', d['ms_per_step'], d['kernel_ms'], d['plan']['plan_seconds']*1e3, d['verified_rows_vs_oracle']))" "$setting"
done
