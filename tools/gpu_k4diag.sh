#!/bin/bash
# K4 diagnosis: the packed-u16 VALU roof on this GPU (tools/micro/pk_rate) and SQ counters of the
# C5 FW kernels (separate --pmc passes, tools/pmc_run.sh)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 60 tools/micro/pk_rate > gpurun_out/pk_rate.txt 2>&1 || { echo pk_rate failed; cat gpurun_out/pk_rate.txt; exit 1; }
cat gpurun_out/pk_rate.txt
BENCH_ARGS="--config c5" bash tools/pmc_run.sh k4 && echo pmc ok
