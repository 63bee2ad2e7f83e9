# device framing: GPU test, then throughput of the product and a variant (GPU box)
set -o pipefail
O=gpurun_out/${TAG:-frame}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_frame.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in http memcache; do
  for lib in libl7gpu.so ${VARLIB:-}; do
    echo "== $lib"; L7G_LIB=$PWD/cilium_amd/$lib timeout -k 10 300 python -u tools/exp_frame.py $k 1000000 16384 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
