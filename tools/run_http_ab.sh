# HTTP A/B (GPU box): every HTTP GPU test on the product, then cfg2 and cfg5
# bench steps alternating the product and the libraries named in LIBS
# (cilium_amd/libl7gpu_<name>.so).   usage: LIBS="old" TAG=x bash tools/run_http_ab.sh
set -o pipefail
O=gpurun_out/${TAG:-httpab}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_http.py tests/test_gpu_http_fast.py tests/test_gpu_http_latency.py tests/test_gpu_nfa.py tests/test_gpu_large_nfa.py tests/test_gpu_cfg4.py tests/test_gpu_envoy_adapter.py tests/test_gpu_service.py tests/test_gpu_streams_mixed.py tests/test_gpu_frame.py tests/test_gpu_proxylib_http_kafka.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; exit 1; }
for wl in cfg2 cfg5; do
  WL=$wl TAG=${TAG:-httpab}/$wl LIBS="prod ${LIBS:-old}" ROUNDS=${ROUNDS:-2} bash tools/ab_libs.sh || exit 2
done
