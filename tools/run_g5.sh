set -o pipefail
# grouped HTTP path: GPU tests, then the cfg4 bench line
O=gpurun_out/g5; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_cfg4.py tests/test_gpu_http.py tests/test_gpu_batcher.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python -u bench.py --workload cfg4 --no-cpu-baseline --no-e2e --no-latency > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -20 $O/bench_cfg4.err; exit 1; }
cat $O/bench_cfg4.json
