set -o pipefail
# memcached A/B (GPU box): the memcached GPU tests on the product library, then
# the mixed stream through the product library and variant builds
O=gpurun_out/mab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_memcache.py tests/test_gpu_proxylib.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
EXP_WORKLOAD=mixed timeout -k 10 500 python -u tools/exp_kafka.py 4000000 ${VARIANTS:-prod} > $O/mixed.log 2>&1 || { cat $O/mixed.log; exit 1; }
cat $O/mixed.log
