# kernel durations of one-request memcached calls (GPU box)
set -o pipefail
O=gpurun_out/${TAG:-ondata}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o prof --output-format csv -- python3 -u $GRAFT_REPO_ROOT/tools/exp_ondata.py > $GRAFT_REPO_ROOT/$O/log.txt 2>&1 || exit 1
grep classify_host $GRAFT_REPO_ROOT/$O/log.txt
cut -d, -f1-4 $GRAFT_REPO_ROOT/$O/prof/prof_kernel_stats.csv | head -8
