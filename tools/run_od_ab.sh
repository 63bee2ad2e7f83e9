# one-request memcached path: kernel time (rocprof), OnData latency, cfg5 (GPU box)
set -o pipefail
TAG=od2 bash tools/ondata_prof.sh || exit 1
ONLY_ZC=1 TAG=od2 bash tools/lat_ab.sh || exit 1
VARS="od0" WLS="cfg5" TAG=od2 TESTS="tests/test_gpu_memcache.py tests/test_gpu_proxylib.py" bash tools/run_ab3.sh || exit 1
