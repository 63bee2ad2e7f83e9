# Round 6, call H (GPU box): service / sync tests on the product, memcached beside Kafka
# (km4 / km5: Kafka on 4 / 5 workgroups per CU) against the product on cfg5, latency leg.
set -o pipefail
O=gpurun_out/r6h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_sync_path.py tests/test_gpu_envoy_adapter.py tests/test_gpu_proxylib.py tests/test_gpu_streams_mixed.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; exit 1; }
TAG=r6h/ab LIBS="prod km5 km4" ROUNDS=2 bash tools/ab_libs.sh || exit 2
timeout -k 10 300 python -u bench.py --workload cfg2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-streams > $O/lat.log 2>&1 || { tail -5 $O/lat.log; exit 3; }
grep '^{' $O/lat.log > $O/lat.json
python3 -c "import json; d=json.load(open('$O/lat.json'))['latency']; print(d['sync_classify_host'], d['proxylib_ondata_memcached'])"
