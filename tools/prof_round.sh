#!/bin/bash
# Profiles for the judged numbers: rocprofv3 kernel-trace stats of the C2/C3/C4 benches and the
# HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) for C3 and C4.
# Outputs under gpurun_out/prof_<tag>/ ; copy the summaries into profiles/ afterwards.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tag=${1:-r01}
mkdir -p gpurun_out/prof_$tag
ks() {  # name bench-args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag/$name -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --verify 0 "$@" > gpurun_out/prof_$tag/$name.json 2> gpurun_out/prof_$tag/$name.err \
    || { echo "kernel trace $name failed"; tail -5 gpurun_out/prof_$tag/$name.err; exit 1; }
}
if [ "${PROF_STATS:-1}" != 0 ]; then  # (PROF_STATS=0: the PMC passes only)
ks c2 --config c2 --steps 20 --warmup 5
ks c3 --config c3 --steps 10 --warmup 2
ks c4 --config c4 --steps 5 --warmup 1
ks c5 --config c5 --steps 5 --warmup 1
ks c3f --config c3f --steps 3 --warmup 1
ks c2f --config c2f --steps 10 --warmup 2
ks c4f --config c4f --steps 2 --warmup 1
fi
pmc() {  # cfg counter bench-args...
  local cfg=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/prof_$tag/pmc_$cfg/$ctr -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --verify 0 "$@" > gpurun_out/prof_$tag/pmc_${cfg}_$ctr.log 2>&1 \
    || { echo "pmc $cfg $ctr failed"; exit 1; }
  cp gpurun_out/prof_$tag/pmc_$cfg/$ctr/run_counter_collection.csv gpurun_out/prof_$tag/pmc_$cfg/$(echo $ctr | tr A-Z a-z | sed 's/_size//')_counter_collection.csv
}
[ "${PROF_PMC:-1}" = 0 ] && { echo prof done; exit 0; }
pmc c2 FETCH_SIZE --config c2 --steps 5 --warmup 2
pmc c2 WRITE_SIZE --config c2 --steps 5 --warmup 2
[ "${PROF_PMC}" = c2 ] && { echo prof done; exit 0; }
pmc c4 FETCH_SIZE --config c4 --steps 2 --warmup 1
pmc c4 WRITE_SIZE --config c4 --steps 2 --warmup 1
pmc c3 FETCH_SIZE --config c3 --steps 2 --warmup 1
pmc c3 WRITE_SIZE --config c3 --steps 2 --warmup 1
pmc c5 FETCH_SIZE --config c5 --steps 3 --warmup 1
pmc c5 WRITE_SIZE --config c5 --steps 3 --warmup 1
pmc c3f FETCH_SIZE --config c3f --steps 2 --warmup 1
pmc c3f WRITE_SIZE --config c3f --steps 2 --warmup 1
pmc c4f FETCH_SIZE --config c4f --steps 1 --warmup 1
pmc c4f WRITE_SIZE --config c4f --steps 1 --warmup 1
echo prof done
