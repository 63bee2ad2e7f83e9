set -o pipefail
# Kafka A/B per request kind of cfg3 (produce / fetch / other)
O=gpurun_out/k5d; mkdir -p $O
for wl in cfg3produce cfg3fetch cfg3other; do
  EXP_WORKLOAD=$wl timeout -k 10 300 python -u tools/exp_kafka.py 1000000 prod ${VARIANTS:-r4} > $O/$wl.log 2>&1 || { cat $O/$wl.log; exit 1; }
  cat $O/$wl.log
done
