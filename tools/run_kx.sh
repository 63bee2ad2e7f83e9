# Kafka layout A/B (GPU box): product vs variant builds, cfg3 and mixed
set -o pipefail
O=gpurun_out/kx; mkdir -p $O
timeout -k 10 300 python -u tools/exp_kafka.py 1000000 prod noxcd cls clsnoxcd > $O/cfg3.log 2>&1 || { cat $O/cfg3.log; exit 1; }
cat $O/cfg3.log
EXP_WORKLOAD=mixed timeout -k 10 400 python -u tools/exp_kafka.py 4000000 prod noxcd cls clsnoxcd > $O/mixed.log 2>&1 || { cat $O/mixed.log; exit 2; }
cat $O/mixed.log
