# large-NFA parity + the kernels the change touched (GPU box)
set -o pipefail
O=gpurun_out/${TAG:-nfa}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_large_nfa.py tests/test_gpu_nfa.py tests/test_gpu_cassandra.py tests/test_gpu_r2d2.py tests/test_gpu_memcache.py > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log; exit $rc
