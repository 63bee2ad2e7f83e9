# Round 6, call P (GPU box): the latency path's well-formed-head shortcut
# (lat_fast): HTTP latency / service / Envoy adapter / fast-path GPU tests,
# then the bench's latency leg (prod) against the previous library (old).
set -o pipefail
O=gpurun_out/${TAG:-r6p}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_http_fast.py tests/test_gpu_http_latency.py tests/test_gpu_service.py tests/test_gpu_envoy_adapter.py tests/test_gpu_sync_path.py tests/test_gpu_http.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; exit 1; }
for v in prod old; do
  if [ $v = prod ]; then L=cilium_amd/libl7gpu.so; else L=cilium_amd/libl7gpu_$v.so; fi
  L7G_LIB=$L timeout -k 10 300 python -u bench.py --workload cfg2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-streams > $O/lat_$v.log 2>&1 || { tail -5 $O/lat_$v.log; exit 3; }
  grep '^{' $O/lat_$v.log > $O/lat_$v.json
  python3 -c "import json; d=json.load(open('$O/lat_$v.json'))['latency']; print('$v', d['sync_classify_host'], d['proxylib_ondata_memcached'])"
done
