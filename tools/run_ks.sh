set -o pipefail
O=gpurun_out/ks; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kafka.py tests/test_gpu_kafka_compressed.py tests/test_gpu_proxylib_http_kafka.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u tools/exp_kafka.py 1000000 prod regs > $O/cfg3.log 2>&1 || { cat $O/cfg3.log; exit 2; }
grep -E "prod|regs" $O/cfg3.log
EXP_WORKLOAD=mixed timeout -k 10 400 python -u tools/exp_kafka.py 8000000 prod regs > $O/mixed.log 2>&1 || { cat $O/mixed.log; exit 3; }
grep -E "prod|regs" $O/mixed.log
