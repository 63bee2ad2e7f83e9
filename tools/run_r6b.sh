# Round 6, call B (GPU box): the overlap test + every GPU test on the product,
# then cfg5 A/B of Kafka/memcached beside HTTP (prod) against one after the
# other (seq), twice each.
set -o pipefail
O=gpurun_out/r6b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
TAG=r6b/ab LIBS="r5 seq prod" ROUNDS=2 bash tools/ab_libs.sh || exit 2
