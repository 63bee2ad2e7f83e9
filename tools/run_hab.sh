set -o pipefail
# cfg2 bench lines alternating the product library and libl7gpu_${VAR}.so
O=gpurun_out/hab; mkdir -p $O
for i in 1 2; do
  for lib in libl7gpu.so libl7gpu_${VAR:-pre}.so; do
    L7G_LIB=$PWD/cilium_amd/$lib timeout -k 10 300 python3 -u bench.py --workload ${WL:-cfg2} --steps 30 --no-cpu-baseline --no-e2e > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
    grep '^{' $O/run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()}, d['parity']['mismatches'])"
  done
done
