# round 4: new GPU tests, fill bench, C5 (K4 fused) bench, KD variant A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_payload_gpu.py tests/test_kf_gpu.py tests/test_topology_gpu.py tests/test_fw_gpu.py tests/test_seed_gpu.py::test_c3_writer_ring_no_stall tests/test_seed_gpu.py::test_c3_eight_rank_plans_every_row} \
  > gpurun_out/r4c_tests.log 2>&1 || { tail -30 gpurun_out/r4c_tests.log; exit 1; }
tail -2 gpurun_out/r4c_tests.log
timeout -k 10 300 python -u tools/fill_bench.py --configs c3,c4 --out gpurun_out/r4_fill.json > gpurun_out/r4_fill.log 2>&1 || { tail -20 gpurun_out/r4_fill.log; exit 1; }
python -c "import json; [print(r['config'], r['layout'], r['fill_s'], r['triangle_bytes'], r['host_write_GBps'], r.get('engine',{}).get('fill_warm_s')) for r in json.load(open('gpurun_out/r4_fill.json'))]"
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --no-cpu-baseline > gpurun_out/r4c_c5.json 2> gpurun_out/r4c_c5.err || { tail gpurun_out/r4c_c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4c_c5.json')); print('C5 K3', d['kernel_ms'], 'FW', d['k4']['fw_table_ms'], 'rows', d['k4']['fw_rows_ms'], d['k4']['rows_verified_vs_oracle'])"
L=SHD_ROUTE_LIB=shadow_amd/libshd_route
bash tools/gpu_ab4.sh ${L}_wcap2ds.so ${L}_fl.so ${L}_flw.so ${L}_lw.so ${L}_icond2.so ${L}_flwi.so ${L}_lwi.so ${L}_wcap2ds.so ${L}_lw.so
CFG=c3 STEPS=30 bash tools/gpu_ab4.sh "SHD_ROUTE_SEEDS=3" "SHD_ROUTE_KDBLOCK=1024" "SHD_ROUTE_KDBLOCK=1024 SHD_ROUTE_SEEDS=3" "SHD_ROUTE_SEED_ROOTS=2048" "SHD_ROUTE_SEED_DEPTH=6" "SHD_ROUTE_FLAGAT=0.5" ${L}_wcap2ds.so ${L}_icond2.so
for v in "SHD_ROUTE_FWREST=1" "SHD_ROUTE_FWREST=0" "SHD_ROUTE_FWREST=3" "SHD_ROUTE_FWREST=3 SHD_ROUTE_FWP=2048" "SHD_ROUTE_FWREST=3 SHD_ROUTE_FWP=512"; do
  env $v timeout -k 10 300 python -u bench.py --config c5 --steps 5 --no-cpu-baseline > gpurun_out/r4c_c5v.json 2> gpurun_out/r4c_c5v.err || { tail gpurun_out/r4c_c5v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r4c_c5v.json')); print('%-40s FW table %.3f ms rows %.3f verified %s' % (sys.argv[1], d['k4']['fw_table_ms'], d['k4']['fw_rows_ms'], d['k4']['rows_verified_vs_oracle']))" "$v"
done
