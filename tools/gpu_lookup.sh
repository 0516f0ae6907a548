#!/bin/bash
# Per-packet lookup bench (tools/lookup_bench.c) on the C2 topology: 1, 4 and 16 threads.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
gcc -O2 -pthread -Iinclude tools/lookup_bench.c -Lshadow_amd -lshd_topology -Wl,-rpath,$PWD/shadow_amd \
    -o gpurun_out/lookup_bench || exit 1
python -c "from shadow_amd import graph; graph.to_graphml(graph.config('c2'), 'gpurun_out/c2.graphml.xml')" || exit 1
for t in 1 4 16; do
    timeout -k 10 120 gpurun_out/lookup_bench gpurun_out/c2.graphml.xml $t 4000000 || exit 1
done
