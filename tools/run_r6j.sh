# Round 6, call J (GPU box): Kafka divergence probe (produce requests of one
# fixed structure vs cfg3's random structure), then the full GPU suite, smoke
# and the cfg5 bench of the product.
set -o pipefail
O=gpurun_out/r6j; mkdir -p $O; export TMPDIR=/tmp
for wl in cfg3produce produni prodcnt; do
  EXP_WORKLOAD=$wl timeout -k 10 240 python -u tools/exp_kafka.py 400000 prod >> $O/div.log 2>&1 || { tail -5 $O/div.log; exit 4; }
done
cat $O/div.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 2; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 3; }
grep '^{' $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v['ms'] for k, v in d['kernels'].items()})"
