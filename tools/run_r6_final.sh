# Round-6 final measurement (GPU box), part 1: smoke, every GPU test, the
# default bench line (CPU baseline, e2e, drop-in latency, streams), rocprof
# kernel statistics and kernel trace (resources) of the same command, then the
# cfg1-cfg4 lines.   usage: TAG=f bash tools/run_r6_final.sh
set -o pipefail
O=gpurun_out/${TAG:-f}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log
[ $rc -ge 124 ] && exit $rc; grep -E "FAILED|ERROR" $O/tests.log | head -20
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
grep '^{' $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()}, d['roofline']['kernel'], d['roofline']['frac'], d['parity'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-latency --no-streams > $O/prof.log 2>&1 || exit 4
python3 tools/kernel_resources.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/kernel_resources.txt; cat $O/kernel_resources.txt
for wl in ${WLS:-cfg1 cfg2 cfg3 cfg4}; do
  timeout -k 10 600 python -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-latency --no-streams > $O/bench_$wl.log 2>&1 || { tail -20 $O/bench_$wl.log; exit 5; }
  grep '^{' $O/bench_$wl.log > $O/bench_$wl.json
  python3 -c "import json; d=json.load(open('$O/bench_$wl.json')); print('$wl', d['ms_per_step'], round(d['value']/1e9,3), d['roofline']['kernel'], d['roofline']['frac'], d['parity']['mismatches'])"
done
echo lines done
