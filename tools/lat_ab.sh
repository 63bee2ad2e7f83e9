# drop-in latency A/B (GPU box): the bench's latency leg with the sync-path switches
set -o pipefail
O=gpurun_out/${TAG:-lat}; mkdir -p $O
run() { timeout -k 10 240 env "$@" python -u -c "import sys, json; sys.path.insert(0, 'tests'); import bench, refpy; from cilium_amd import gen; print(json.dumps(bench.latency_leg(gen, refpy)))"; }
run L7G_SYNC_ZEROCOPY=1 > $O/lat_zc.json 2> $O/lat_zc.err || exit 1
[ -n "$ONLY_ZC" ] || run L7G_SYNC_ZEROCOPY=0 > $O/lat_copy.json 2> $O/lat_copy.err || exit 1
for f in $O/lat_*.json; do echo "== $f"; python3 -c "
import json,sys; d=json.load(open('$f'))
print('sync', d['sync_classify_host']['p50_us'], d['sync_classify_host']['p99_us'], 'ondata', d['proxylib_ondata_memcached']['p50_us'], d['proxylib_ondata_memcached']['p99_us'])
for b in d['batcher']: print('  batcher', b['offered_per_s'], b['max_requests'], 'achieved', round(b['achieved_per_s']), 'p50', b['latency']['p50_us'], 'p99', b['latency']['p99_us'])
"; done
