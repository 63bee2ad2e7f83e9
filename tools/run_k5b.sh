set -o pipefail
# Kafka A/B (cfg3 and mixed) of the product and variant builds, no tests
O=gpurun_out/k5b; mkdir -p $O
timeout -k 10 400 python -u tools/exp_kafka.py 1000000 prod ${VARIANTS:-r4} > $O/cfg3.log 2>&1 || { cat $O/cfg3.log; exit 1; }
cat $O/cfg3.log
EXP_WORKLOAD=mixed timeout -k 10 400 python -u tools/exp_kafka.py 4000000 prod ${VARIANTS:-r4} > $O/mixed.log 2>&1 || { cat $O/mixed.log; exit 1; }
cat $O/mixed.log
