# Round 6, call K (GPU box): produce requests through the flat message loop:
# Kafka GPU tests, then cfg3 and cfg5 A/B against the previous kernel (old).
set -o pipefail
O=gpurun_out/r6k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kafka_flat.py tests/test_gpu_kafka.py tests/test_gpu_kafka_compressed.py tests/test_kafka_wire_kats.py tests/test_gpu_proxylib_http_kafka.py tests/test_gpu_streams_mixed.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; exit 1; }
EXP_WORKLOAD=cfg3 timeout -k 10 300 python -u tools/exp_kafka.py 2000000 prod old > $O/cfg3.log 2>&1 || { tail -5 $O/cfg3.log; exit 4; }
grep -v Warn $O/cfg3.log | grep -E "prod|old|requests"
TAG=r6k/ab LIBS="prod old" ROUNDS=2 bash tools/ab_libs.sh || exit 2
