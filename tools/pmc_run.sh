#!/bin/bash
# Separate rocprofv3 --pmc passes (one counter group per run, never combined with
# tracing) over a short bench.py run; CSVs land in gpurun_out/pmc_<tag>/.
# usage: tools/pmc_run.sh <tag> <bench args...>
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/pmc_${tag}/${name} -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify 0 $BENCH_ARGS > gpurun_out/pmc_${tag}/${name}.log 2>&1
}
mkdir -p gpurun_out/pmc_${tag}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
echo pmc done
