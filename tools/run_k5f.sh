set -o pipefail
# Kafka phase timing (cfg3produce / cfg3), then PMC of three builds on cfg3produce
O=gpurun_out/k5f; mkdir -p $O
VARIANTS="ph nocrc r4" bash tools/run_k5e.sh || exit 1
for v in prod nocrc r4; do
  EXP_WORKLOAD=cfg3produce timeout -k 10 600 bash tools/pmc_run.sh $O/pmc_$v python -u tools/exp_kafka.py 500000 $v > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
  python tools/pmc_summary.py $O/pmc_$v kafka_classify > $O/pmc_$v.txt
  echo "== $v"; cat $O/pmc_$v.txt
done
