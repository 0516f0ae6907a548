#!/bin/bash
# K4 A/B: rocprofv3 kernel stats of the C5 bench with the 64x64 rest kernel (FWREST=1) and the
# 128x128-region one (default), FW table time from the bench line of each
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fwab
for v in 1 2; do
  SHD_ROUTE_FWREST=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/fwab/v$v -o run --output-format csv \
    -- python3 bench.py --config c5 --no-cpu-baseline --verify 0 --steps 5 --warmup 1 > gpurun_out/fwab/v$v.json 2> gpurun_out/fwab/v$v.err \
    || { echo "v$v failed"; tail -5 gpurun_out/fwab/v$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/fwab/v$v.json').read().strip().splitlines()[-1]);print('v$v fw', d['k4']['fw_table_ms'])"
  f=$(find gpurun_out/fwab/v$v -name "*kernel_stats.csv" | head -1)
  grep -E "fw_" "$f" | cut -d, -f1-4
done
if [ "${PLANDBG:-1}" = 1 ]; then
SHD_ROUTE_PLAN_DEBUG=1 timeout -k 10 240 python3 bench.py --no-cpu-baseline --verify 0 --steps 3 --warmup 1 > gpurun_out/fwab/c4.json 2> gpurun_out/fwab/c4.err || { echo c4 failed; exit 1; }
grep -E "closeness|plan total" gpurun_out/fwab/c4.err
fi
