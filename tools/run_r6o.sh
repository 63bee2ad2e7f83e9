# Round 6, call O (GPU box): Kafka kernel at 7 waves per SIMD (448-thread
# workgroups, 72 VGPRs: w7) against the product (6 waves): cfg3 and cfg5.
set -o pipefail
O=gpurun_out/r6o; mkdir -p $O; export TMPDIR=/tmp
EXP_WORKLOAD=cfg3 timeout -k 10 300 python -u tools/exp_kafka.py 4000000 prod w7 > $O/cfg3.log 2>&1 || { tail -5 $O/cfg3.log; exit 4; }
grep -E "prod|w7|requests" $O/cfg3.log
TAG=r6o/ab LIBS="prod w7" ROUNDS=2 bash tools/ab_libs.sh || exit 2
