# Round 6, call L (GPU box): flat produce loop with 64-byte aligned blocks:
# Kafka GPU tests, then cfg3 and cfg5 A/B against the previous kernel (old).
set -o pipefail
O=gpurun_out/${TAG:-r6l}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kafka_flat.py tests/test_gpu_kafka.py tests/test_gpu_kafka_compressed.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; exit 1; }
for wl in cfg3 cfg3produce; do
EXP_WORKLOAD=$wl timeout -k 10 300 python -u tools/exp_kafka.py 4000000 prod old > $O/$wl.log 2>&1 || { tail -5 $O/$wl.log; exit 4; }
grep -v Warn $O/$wl.log | grep -E "prod|old|requests"
done
TAG=${TAG:-r6l}/ab LIBS="prod old" ROUNDS=1 bash tools/ab_libs.sh || exit 2
