# Round measurement set (GPU box): smoke, all GPU tests, default bench, rocprof stats, cfg1-4 lines
set -o pipefail
O=gpurun_out/${TAG:-final}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit 3
grep '^{' $O/bench.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/prof.log 2>&1 || exit 4
for w in cfg1 cfg2 cfg3 cfg4; do
  timeout -k 10 600 python -u bench.py --workload $w --steps 20 --warmup 5 > $O/bench_$w.log 2>&1 || exit 5
done
echo done
