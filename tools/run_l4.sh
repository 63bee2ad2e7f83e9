set -o pipefail
O=gpurun_out/l4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_http.py tests/test_gpu_nfa.py tests/test_gpu_cfg4.py tests/test_gpu_unowned.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u tools/exp_mixed.py 8000000 > $O/mx_prod.log 2>&1 || exit 2
EXP_LIB=libl7gpu_lane1.so timeout -k 10 300 python -u tools/exp_mixed.py 8000000 > $O/mx_lane1.log 2>&1 || exit 3
grep "ms/step" $O/mx_prod.log $O/mx_lane1.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/cfg5.log 2>&1 || exit 4
grep -o '"kernels": {[^}]*}[^}]*}[^}]*}[^}]*}' $O/cfg5.log | head -2
