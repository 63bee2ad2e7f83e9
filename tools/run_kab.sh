set -o pipefail
# Kafka A/B: product library vs variant builds, cfg3 and mixed, then the Kafka GPU tests
O=gpurun_out/kab; mkdir -p $O
timeout -k 10 400 python -u tools/exp_kafka.py 1000000 ${VARIANTS:-prod} > $O/cfg3.log 2>&1 || { cat $O/cfg3.log; exit 1; }
cat $O/cfg3.log
EXP_WORKLOAD=mixed timeout -k 10 400 python -u tools/exp_kafka.py 4000000 ${VARIANTS:-prod} > $O/mixed.log 2>&1 || { cat $O/mixed.log; exit 1; }
cat $O/mixed.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kafka.py tests/test_gpu_kafka_compressed.py tests/test_kafka_wire_kats.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
