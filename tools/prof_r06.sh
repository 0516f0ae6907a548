#!/bin/bash
# Round-6 profiles of the shipped build: rocprofv3 kernel-trace stats and the HBM PMC passes
# (FETCH_SIZE / WRITE_SIZE in separate runs) for the BASELINE configs, summarised on the box
# per kernel with the build id bench.py prints (tools/pmc_traffic.py), so a bench line only
# takes counter bytes of its own kernel and build.   usage: TAG=r06 CFGS="c4 c3 c2 c5" bash tools/prof_r06.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tag=${TAG:-r06}; mkdir -p gpurun_out/prof_$tag
ks() { local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag/$name -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --verify 0 "$@" > gpurun_out/prof_$tag/$name.json 2> gpurun_out/prof_$tag/$name.err \
    || { echo "kernel trace $name failed"; tail -5 gpurun_out/prof_$tag/$name.err; exit 1; }
  cp gpurun_out/prof_$tag/$name/run_kernel_stats.csv gpurun_out/${tag}_kernel_stats_$name.csv 2>/dev/null || \
    find gpurun_out/prof_$tag/$name -name "*kernel_stats.csv" -exec cp {} gpurun_out/${tag}_kernel_stats_$name.csv \; ; }
pmc() { local cfg=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/prof_$tag/pmc_$cfg/$ctr -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --verify 0 "$@" > gpurun_out/prof_$tag/pmc_${cfg}_$ctr.log 2>&1 \
    || { echo "pmc $cfg $ctr failed"; exit 1; }
  f=$(find gpurun_out/prof_$tag/pmc_$cfg/$ctr -name "*counter_collection.csv" | head -1)
  cp "$f" gpurun_out/prof_$tag/pmc_$cfg/$(echo $ctr | tr A-Z a-z | sed 's/_size//')_counter_collection.csv; }
for cfg in ${CFGS:-c4 c3 c2 c5}; do
  case $cfg in
    c4) a="--config c4 --steps 5 --warmup 1"; p="--config c4 --steps 2 --warmup 1"; s=50000; k=sssp_delta_kernel ;;
    c3) a="--config c3 --steps 10 --warmup 2"; p="--config c3 --steps 2 --warmup 1"; s=9337; k="" ;;
    c2) a="--config c2 --steps 20 --warmup 5"; p="--config c2 --steps 5 --warmup 2"; s=2000; k="" ;;
    c5) a="--config c5 --steps 5 --warmup 1"; p="--config c5 --steps 3 --warmup 1"; s=4000; k="" ;;
    c3f) a="--config c3f --steps 3 --warmup 1"; p="--config c3f --steps 2 --warmup 1"; s=9337; k="" ;;
    c2f) a="--config c2f --steps 10 --warmup 2"; p="--config c2f --steps 3 --warmup 1"; s=2000; k="" ;;
    c4f) a="--config c4f --steps 2 --warmup 1"; p="--config c4f --steps 1 --warmup 1"; s=50000; k="" ;;
  esac
  ks $cfg $a || exit 1
  pmc $cfg FETCH_SIZE $p && pmc $cfg WRITE_SIZE $p || exit 1
  python3 tools/pmc_traffic.py gpurun_out/prof_$tag/pmc_$cfg gpurun_out/${tag}_pmc_$cfg.json $cfg $s $k > /dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/${tag}_pmc_$cfg.json'));print('$cfg', d['build_id'], {k: round((v['fetch_bytes']+v['write_bytes'])/1e9,3) for k,v in d['kernels'].items()})"
done
echo prof done
