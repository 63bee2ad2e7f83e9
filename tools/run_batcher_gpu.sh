# batcher parity + latency leg on the GPU box
set -o pipefail
O=gpurun_out/${TAG:-bat}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_batcher.py tests/test_gpu_envoy_adapter.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
ONLY_ZC=1 TAG=${TAG:-bat} bash tools/lat_ab.sh
