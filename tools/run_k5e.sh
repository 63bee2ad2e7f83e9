set -o pipefail
# Kafka A/B on cfg3 only (produce-only and whole), no tests
O=gpurun_out/k5e; mkdir -p $O
for wl in cfg3produce cfg3; do
  EXP_WORKLOAD=$wl timeout -k 10 300 python -u tools/exp_kafka.py 1000000 prod ${VARIANTS:-r4} > $O/$wl.log 2>&1 || { cat $O/$wl.log; exit 1; }
  grep -v "Warning\|from_numpy\|amdgpu.ids" $O/$wl.log
done
