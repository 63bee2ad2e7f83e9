# A/B on the GPU box: selected GPU tests with the product library, then bench
# lines alternating the product and libl7gpu_${VAR}.so on each workload.
# usage: TAG=x VARS="nofast other" WLS="cfg5 cfg2" TESTS="tests/a.py ..." bash tools/run_ab3.sh
set -o pipefail
O=gpurun_out/${TAG:-ab3}; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for wl in ${WLS:-cfg5}; do
  for i in 1 2; do
    for lib in libl7gpu.so $(for v in ${VARS:-nofast}; do echo libl7gpu_$v.so; done); do
      L7G_LIB=$PWD/cilium_amd/$lib timeout -k 10 300 python3 -u bench.py --workload $wl --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-e2e --no-latency > $O/run_${wl}.log 2>&1 || { tail -20 $O/run_${wl}.log; exit 2; }
      grep '^{' $O/run_${wl}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl', '$lib', d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()}, d['parity']['mismatches'])"
    done
  done
done
echo done
