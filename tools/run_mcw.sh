set -o pipefail
O=gpurun_out/mcw; mkdir -p $O
EXP_WORKLOAD=mixed timeout -k 10 400 python -u tools/exp_kafka.py 8000000 prod mcw7 mcw8 > $O/mixed.log 2>&1 || { cat $O/mixed.log; exit 2; }
cat $O/mixed.log
