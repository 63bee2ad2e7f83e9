# Round-4 GPU check: smoke, every GPU test, the default bench line (CPU
# baseline, e2e, drop-in latency).  usage: TAG=x bash tools/run_r4.sh
set -o pipefail
O=gpurun_out/${TAG:-r4}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log
[ $rc -ge 124 ] && exit $rc
grep -E "FAILED|ERROR" $O/tests.log | head -20
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
grep '^{' $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()}, d['roofline']['kernel'], d['roofline']['frac'], d['parity']); print(json.dumps(d.get('latency'))[:1500])"
echo done
