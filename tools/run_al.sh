set -o pipefail
O=gpurun_out/al; mkdir -p $O
timeout -k 10 300 python -u tools/exp_mixed.py 8000000 > $O/mx_prod.log 2>&1 || exit 2
EXP_LIB=libl7gpu_w128.so timeout -k 10 300 python -u tools/exp_mixed.py 8000000 > $O/mx_w128.log 2>&1 || exit 3
grep "ms/step" $O/mx_prod.log $O/mx_w128.log
