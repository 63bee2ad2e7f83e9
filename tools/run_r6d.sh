# Round 6, call D (GPU box): HTTP kernel occupancy variants (waves per
# workgroup, window bytes, map depth) on cfg5 and cfg2, twice each.
set -o pipefail
O=gpurun_out/r6d; mkdir -p $O; export TMPDIR=/tmp
TAG=r6d/cfg5 LIBS="prod h16d1 h16d2 h12d2 h8d2" ROUNDS=1 bash tools/ab_libs.sh || exit 2
TAG=r6d/cfg2 WL=cfg2 STEPS=20 LIBS="prod h16d1 h16d2 h12d2 h8d2" ROUNDS=1 bash tools/ab_libs.sh || exit 3
