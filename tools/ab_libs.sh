# A/B of library builds on one box (GPU box): the cfg5 bench step through each
# library in LIBS (product = libl7gpu.so), alternating ROUNDS times, with the
# per-kernel HIP-event times.  usage: LIBS="r5 prod mcw4" WL=cfg5 bash tools/ab_libs.sh
set -o pipefail
O=gpurun_out/${TAG:-ab}; mkdir -p $O
for r in $(seq 1 ${ROUNDS:-1}); do
for v in ${LIBS:-prod}; do
  if [ $v = prod ]; then L=cilium_amd/libl7gpu.so; else L=cilium_amd/libl7gpu_$v.so; fi
  L7G_LIB=$L timeout -k 10 300 python -u bench.py --workload ${WL:-cfg5} --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-e2e --no-latency --no-streams $EXTRA > $O/${v}_$r.log 2>&1 || { tail -5 $O/${v}_$r.log; exit 1; }
  grep '^{' $O/${v}_$r.log > $O/${v}_$r.json
  python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v', '$r', round(d['ms_per_step'],3), {k:round(v['ms'],3) for k,v in d['kernels'].items()}, d['parity']['mismatches'])"
done
done
