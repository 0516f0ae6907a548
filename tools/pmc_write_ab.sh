#!/bin/bash
# WRITE_SIZE per C4 launch for alternative engine libraries (A/B of write traffic):
#   bash tools/pmc_write_ab.sh shadow_amd/libshd_route.so shadow_amd/libshd_route_alt.so ...
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_ab
i=0
for lib in "$@"; do
  i=$((i+1))
  SHD_ROUTE_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_ab/w$i -o run --output-format csv \
    -- python3 bench.py --config ${CFG:-c4} --steps 1 --warmup 0 --no-cpu-baseline --verify 0 > gpurun_out/pmc_ab/w$i.log 2>&1 || { echo "pass $lib failed"; exit 1; }
  python3 - "$lib" gpurun_out/pmc_ab/w$i/run_counter_collection.csv <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) * 1024 / 1e9 for r in csv.DictReader(open(sys.argv[2])) if "sssp_" in r["Kernel_Name"]]
print(sys.argv[1], "WRITE GB per launch", [round(x, 2) for x in v])
PY
done
