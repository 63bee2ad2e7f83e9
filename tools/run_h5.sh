set -o pipefail
# HTTP A/B (GPU box): tests, then exp_http rows on the product and the base build
O=gpurun_out/h5; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_http.py tests/test_gpu_http_latency.py tests/test_gpu_cfg4.py tests/test_gpu_nfa.py tests/test_gpu_envoy_adapter.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in prod base prod base; do
  if [ $v = prod ]; then L=; else L=libl7gpu_$v.so; fi
  EXP_LIB=$L timeout -k 10 300 python -u tools/exp_http.py 1000000 ${ROWS:-a,d,e,f,g,h} 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 2
done
