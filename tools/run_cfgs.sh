set -o pipefail
# bench lines for cfg1-cfg4 (GPU box), no CPU baseline / e2e legs
O=gpurun_out/cfgs; mkdir -p $O
for wl in cfg1 cfg2 cfg3 cfg4; do
  timeout -k 10 300 python3 -u bench.py --workload $wl --no-cpu-baseline --no-e2e > $O/$wl.log 2>&1 || { tail -20 $O/$wl.log; exit 1; }
  grep '^{' $O/$wl.log > $O/$wl.json
  python3 -c "import json; d=json.load(open('$O/$wl.json')); print('$wl', d['ms_per_step'], round(d['value']/1e9,3), d['roofline']['kernel'], d['roofline']['frac'], d['parity']['mismatches'])"
done
