# Multi-GPU partition sweep: every rank of a W-way strong split run in turn on this GPU,
# per env variant ("" = default), e.g.
#   CFG=c3 W="1 8" bash tools/gpu_emul_sweep.sh "" "SHD_ROUTE_SEED_DEPTH=2"
# Each variant's log: gpurun_out/emul_${TAG}_<i>.log (TAG defaults to the config).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CFG=${CFG:-c4}
W=${W:-8}
TAG=${TAG:-$CFG}
REPS=${REPS:-2}
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== [$v]"
  env $v timeout -k 10 ${TLIM:-200} python -u tools/emul_ranks.py --config $CFG --world $W --reps $REPS \
      > gpurun_out/emul_${TAG}_$i.log 2>&1 || { echo "variant [$v] failed"; tail -5 gpurun_out/emul_${TAG}_$i.log; exit 1; }
  grep -E "^W=[0-9]+:" gpurun_out/emul_${TAG}_$i.log
done
