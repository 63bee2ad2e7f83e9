set -o pipefail
# memcached A/B (GPU box): entry fields carried from the kind pass (prod) vs
# fetched again by the classifying lane (base); tests, times, FETCH_SIZE
O=gpurun_out/mc5; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_memcache.py tests/test_gpu_proxylib.py tests/test_gpu_sync_path.py tests/test_gpu_unowned.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
EXP_WORKLOAD=mc timeout -k 10 300 python -u tools/exp_kafka.py 4000000 prod base prod base > $O/mc.log 2>&1 || { cat $O/mc.log; exit 1; }
cat $O/mc.log
EXP_WORKLOAD=mixed timeout -k 10 500 python -u tools/exp_kafka.py 4000000 prod base prod base > $O/mixed.log 2>&1 || { cat $O/mixed.log; exit 1; }
cat $O/mixed.log
for v in prod base; do
  EXP_WORKLOAD=mc timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f_$v -o pmc --output-format csv -- python3 -u tools/exp_kafka.py 4000000 $v > $O/f_$v.log 2>&1 || exit 4
  python3 tools/pmc_summary.py $O/f_$v memcache_classify | sed "s/^/$v /"
done
