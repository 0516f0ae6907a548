#!/bin/bash
# Round-end GPU call: every -m gpu test, smoke, then one bench line per config (C4 the driver
# default with CPU baselines; C5 with its CPU baselines; C3, C2, C3f, C2f without).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
tag=${TAG:-r3final}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_$tag.log | tail -30; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
timeout -k 10 180 python -u __graft_entry__.py smoke || exit 1
SHD_ROUTE_PLAN_DEBUG=1 timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_${tag}_c4.json 2> gpurun_out/bench_${tag}_c4.err || { echo BENCH C4 FAILED; tail gpurun_out/bench_${tag}_c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 > gpurun_out/bench_${tag}_c5.json 2> gpurun_out/bench_${tag}_c5.err || { echo BENCH C5 FAILED; tail gpurun_out/bench_${tag}_c5.err; exit 1; }
for c in c3 c2 c3f c2f; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${tag}_$c.json 2> gpurun_out/bench_${tag}_$c.err || { echo BENCH $c FAILED; tail gpurun_out/bench_${tag}_$c.err; exit 1; }
done
python - <<PY
import json
for c in ["c4", "c5", "c3", "c2", "c3f", "c2f"]:
    d = json.load(open(f"gpurun_out/bench_${tag}_{c}.json"))
    print(c, round(d["value"]), "ms/step", round(d["ms_per_step"], 4), "frac", round(d["roofline"]["frac"], 4),
          "verified", d.get("verified_rows_vs_oracle"), "ttt", d.get("time_to_table_ms"))
PY
