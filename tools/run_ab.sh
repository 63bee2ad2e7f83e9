set -o pipefail
# A/B (GPU box): GPU parity tests on the product library, then cfg3 and the
# mixed stream through the product library and variant builds (VARIANTS)
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/exp_kafka.py 1000000 ${VARIANTS:-prod} > $O/cfg3.log 2>&1 || { cat $O/cfg3.log; exit 1; }
cat $O/cfg3.log
EXP_WORKLOAD=mixed timeout -k 10 500 python -u tools/exp_kafka.py 4000000 ${VARIANTS:-prod} > $O/mixed.log 2>&1 || { cat $O/mixed.log; exit 1; }
cat $O/mixed.log
