# Round 6, call Q (GPU box): the full GPU suite with lat_fast, then the bench's
# latency leg on one box, product vs the previous library (old: loaded by the
# native latency driver through LD_LIBRARY_PATH), alternating twice.
set -o pipefail
O=gpurun_out/${TAG:-r6q}; mkdir -p $O $O/oldlib; export TMPDIR=/tmp
cp cilium_amd/libl7gpu_old.so $O/oldlib/libl7gpu.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; exit 1; }
for r in 1 2; do
for v in prod old; do
  if [ $v = prod ]; then LP=""; else LP="$PWD/$O/oldlib"; fi
  LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 300 python -u bench.py --workload cfg2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-streams > $O/lat_${v}_$r.log 2>&1 || { tail -5 $O/lat_${v}_$r.log; exit 3; }
  grep '^{' $O/lat_${v}_$r.log > $O/lat_${v}_$r.json
  python3 -c "import json; d=json.load(open('$O/lat_${v}_$r.json'))['latency']; print('$v $r', d['sync_classify_host'], d['proxylib_ondata_memcached'])"
done
done
rm -rf $O/oldlib
