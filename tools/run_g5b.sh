set -o pipefail
# work-counter grab size A/B (GPU box): 1 (prod), 2, 4 tiles / 64-entry groups per atomic
O=gpurun_out/g5b; mkdir -p $O
for v in prod g2 g4 prod g2 g4; do
  if [ $v = prod ]; then L=; else L=libl7gpu_$v.so; fi
  EXP_LIB=$L timeout -k 10 300 python -u tools/exp_http.py 4000000 a,f 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 2
done
EXP_WORKLOAD=cfg3 timeout -k 10 300 python -u tools/exp_kafka.py 1000000 prod g2 g4 prod g2 g4 2>&1 | grep -v amdgpu || exit 3
for v in prod g2 g4 prod g2 g4; do
  if [ $v = prod ]; then export L7G_LIB=; else export L7G_LIB=$PWD/cilium_amd/libl7gpu_$v.so; fi
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-e2e --no-latency --no-streams > $O/b_$v.json 2>/dev/null || exit 4
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); print('$v', d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['parity']['mismatches'])"
done
