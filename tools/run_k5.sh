set -o pipefail
# Kafka round-5 A/B: the Kafka GPU tests on the product build, then cfg3 and
# mixed kernel times of the product vs the round-4 build (libl7gpu_r4.so)
O=gpurun_out/k5; mkdir -p $O
timeout -k 10 120 tools/microbench/crc_lds_bench 2 > $O/crc.log 2>&1 || { cat $O/crc.log; exit 1; }
cat $O/crc.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kafka.py tests/test_gpu_kafka_compressed.py tests/test_kafka_wire_kats.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u tools/exp_kafka.py 1000000 prod ${VARIANTS:-r4} > $O/cfg3.log 2>&1 || { cat $O/cfg3.log; exit 1; }
cat $O/cfg3.log
EXP_WORKLOAD=mixed timeout -k 10 400 python -u tools/exp_kafka.py 4000000 prod ${VARIANTS:-r4} > $O/mixed.log 2>&1 || { cat $O/mixed.log; exit 1; }
cat $O/mixed.log
