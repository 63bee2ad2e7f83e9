# kernel durations of the sync probe (GPU box)
set -o pipefail
O=gpurun_out/${TAG:-probe}; mkdir -p $O
bash tools/sync_probe.sh > $O/probe.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- $GRAFT_REPO_ROOT/tools/experiments/sync_probe block < $GRAFT_REPO_ROOT/$O/in.txt > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" -exec cat {} \;
