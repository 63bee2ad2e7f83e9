set -o pipefail
# latency path: latency_main (Allowed() / OnData one request per call) + the drop-in GPU tests
O=gpurun_out/l5; mkdir -p $O
export PYTHONPATH=$PWD/tests:$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_http_latency.py tests/test_gpu_http.py tests/test_gpu_sync_path.py tests/test_gpu_envoy_adapter.py tests/test_gpu_proxylib.py tests/test_gpu_batcher.py tests/test_gpu_threads.py tests/test_gpu_proxylib_http_kafka.py tests/test_gpu_unowned.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u -c "
import sys, json
import bench, refpy
from cilium_amd import gen
print(json.dumps(bench.latency_leg(gen, refpy, iters=4000)))
" > $O/lat.json 2> $O/lat.err || { tail -20 $O/lat.err; exit 1; }
cat $O/lat.json
if [ "${TRACE:-0}" = 1 ]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o lat -- python3 -u -c "
import sys, json
sys.path[:0] = ['$GRAFT_REPO_ROOT', '$GRAFT_REPO_ROOT/tests']
import bench, refpy
from cilium_amd import gen
print(json.dumps(bench.latency_leg(gen, refpy, iters=300))[:300])
" > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/kt.log; exit 1; }
fi
timeout -k 10 200 python -u tools/exp_lat.py > $O/exp_lat.log 2>&1 || { tail -20 $O/exp_lat.log; exit 1; }
grep -v amdgpu.ids $O/exp_lat.log
L7G_LIB=$PWD/cilium_amd/libl7gpu_ph.so timeout -k 10 200 python -u tools/exp_lat.py > $O/exp_lat_ph.log 2>&1 || { tail -20 $O/exp_lat_ph.log; exit 1; }
grep -v amdgpu.ids $O/exp_lat_ph.log
