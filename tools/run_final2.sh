# Round-end measurement (GPU box): smoke, GPU tests, default bench, rocprof stats, traffic PMC for cfg5/cfg2/cfg3
set -o pipefail
O=gpurun_out/${TAG:-final2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/prof.log 2>&1 || exit 4
for wl in cfg5 cfg2 cfg3; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 170 rocprofv3 --pmc $c -d $O/${wl}_$c -o pmc --output-format csv -- python3 -u bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --profile-steps 0 > $O/${wl}_$c.log 2>&1 || exit 5
  done
done
echo done
