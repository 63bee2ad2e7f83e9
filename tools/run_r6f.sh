# Round 6, call F (GPU box): the service tests, then the latency leg with the services on and off.
set -o pipefail
O=gpurun_out/r6f; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_sync_path.py tests/test_gpu_envoy_adapter.py tests/test_gpu_proxylib.py -x -v --timeout 120 --timeout-method thread > $O/svc_tests.log 2>&1; rc=$?
tail -3 $O/svc_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/svc_tests.log | head -30; exit 1; }
for svc in 1 0 1; do
  L7G_SERVICE=$svc timeout -k 10 300 python -u bench.py --workload cfg2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-streams > $O/lat_svc$svc.log 2>&1 || { tail -5 $O/lat_svc$svc.log; exit 3; }
  grep '^{' $O/lat_svc$svc.log > $O/lat_svc$svc.json
  python3 -c "import json; d=json.load(open('$O/lat_svc$svc.json'))['latency']; print('svc=$svc', d['sync_classify_host'], d['proxylib_ondata_memcached'])"
done
