set -o pipefail
# latency A/B (GPU box): the bench latency leg with the product library and a
# variant swapped in under its name (this is the box's scratch copy of the tree)
cp cilium_amd/libl7gpu.so /tmp/l7_prod.so
for v in prod ${VAR:-h} prod ${VAR:-h}; do
  if [ $v = prod ]; then cp /tmp/l7_prod.so cilium_amd/libl7gpu.so; else cp cilium_amd/libl7gpu_$v.so cilium_amd/libl7gpu.so; fi
  timeout -k 10 300 python -u -c "
import sys, json
sys.path[:0] = ['.', 'tests']
import bench, refpy
from cilium_amd import gen
d = bench.latency_leg(gen, refpy, iters=4000)
print('$v', 'sync', d['sync_classify_host']['p50_us'], 'ondata', d['proxylib_ondata_memcached']['p50_us'])
" 2>/dev/null | grep -E "^[a-z0-9]+ sync" || exit 2
done
cp /tmp/l7_prod.so cilium_amd/libl7gpu.so
