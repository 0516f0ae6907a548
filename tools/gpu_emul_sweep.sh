# Multi-GPU partition sweep: every rank of a W-way strong split run in turn on this GPU,
# per env variant ("" = default), e.g.  bash tools/gpu_emul_sweep.sh "" "SHD_ROUTE_TOPCAP=8"
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CFG=${CFG:-c4}
W=${W:-8}
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== [$v]"
  env $v timeout -k 10 150 python -u tools/emul_ranks.py --config $CFG --world $W --reps 2 \
      > gpurun_out/emul_$i.log 2>&1 || { echo "variant [$v] failed"; tail -5 gpurun_out/emul_$i.log; exit 1; }
  tail -1 gpurun_out/emul_$i.log
done
