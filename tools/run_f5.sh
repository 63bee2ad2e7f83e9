set -o pipefail
# device framing: GPU tests, then throughput per protocol (1M requests, 16k streams)
O=gpurun_out/f5; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_frame.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in http memcache kafka; do
  L7G_LIB=${FLIB:-} timeout -k 10 300 python -u tools/exp_frame.py $k 1000000 16384 > $O/tp_$k.log 2>&1 || { cat $O/tp_$k.log; exit 1; }
  grep -v amdgpu.ids $O/tp_$k.log
done
