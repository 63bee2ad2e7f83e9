set -o pipefail
O=gpurun_out/kv; mkdir -p $O
timeout -k 10 400 python -u tools/exp_kafka.py 1000000 ${VARIANTS:-prod} > $O/cfg3.log 2>&1 || { cat $O/cfg3.log; exit 1; }
cat $O/cfg3.log
