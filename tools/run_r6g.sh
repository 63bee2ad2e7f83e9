# Round 6, call G (GPU box): partition without the Kafka api-key reads (nokey) against the product, cfg5 and cfg3.
set -o pipefail
O=gpurun_out/r6g; mkdir -p $O; export TMPDIR=/tmp
TAG=r6g/cfg5 LIBS="prod nokey" ROUNDS=2 bash tools/ab_libs.sh || exit 2
TAG=r6g/cfg3 WL=cfg3 STEPS=20 LIBS="prod nokey" ROUNDS=2 bash tools/ab_libs.sh || exit 3
