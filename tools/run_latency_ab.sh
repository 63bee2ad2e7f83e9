# Latency A/B (GPU box): the HTTP latency / fast-path / service / Envoy GPU tests,
# the phase split of one-request calls (tools/exp_lat.py with the timing build),
# then the bench latency leg alternating product and cilium_amd/libl7gpu_old.so.
# (Needs cilium_amd/libl7gpu_timing.so: python -m cilium_amd.build --timing, and the
# library to compare against copied to cilium_amd/libl7gpu_old.so.)
set -o pipefail
O=gpurun_out/${TAG:-latab}; mkdir -p $O $O/oldlib; export TMPDIR=/tmp
cp cilium_amd/libl7gpu_old.so $O/oldlib/libl7gpu.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_http_fast.py tests/test_gpu_http_latency.py tests/test_gpu_service.py tests/test_gpu_envoy_adapter.py tests/test_gpu_sync_path.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; exit 1; }
L7G_LIB=cilium_amd/libl7gpu_timing.so timeout -k 10 200 python -u tools/exp_lat.py > $O/lat_timing.log 2>&1 || { tail -5 $O/lat_timing.log; exit 2; }
grep -v amdgpu.ids $O/lat_timing.log
for r in 1 2; do
for v in prod old; do
  if [ $v = prod ]; then LP=""; else LP="$PWD/$O/oldlib"; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 300 python -u bench.py --workload cfg2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-streams > $O/lat_${v}_$r.log 2>&1 || { tail -5 $O/lat_${v}_$r.log; exit 3; }
  grep '^{' $O/lat_${v}_$r.log > $O/lat_${v}_$r.json
  python3 -c "import json; d=json.load(open('$O/lat_${v}_$r.json'))['latency']; print('$v $r', d['sync_classify_host'], d['proxylib_ondata_memcached'])"
done
done
rm -rf $O/oldlib
