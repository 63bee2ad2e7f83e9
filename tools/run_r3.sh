# Round-3 measurement (GPU box): GPU tests, default bench, rocprof kernel stats,
# then the PMC passes of tools/pmc_run.sh over one cfg5 step.
# usage: TAG=r3a [TESTS=0] [PMC=0] bash tools/run_r3.sh
set -o pipefail
O=gpurun_out/${TAG:-r3}; mkdir -p $O; export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  tail -3 $O/tests.log
  [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/tests.log | head -20; exit $rc; }
fi
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()}, d['roofline'], d['parity'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/prof.log 2>&1 || exit 4
if [ "${PMC:-1}" = 1 ]; then
  bash tools/pmc_run.sh $O/pmc python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --profile-steps 0 || exit 5
fi
echo done
