set -o pipefail
O=gpurun_out/${TAG:-h2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_http.py tests/test_gpu_nfa.py tests/test_gpu_cfg4.py tests/test_gpu_unowned.py tests/test_gpu_envoy_adapter.py tests/test_gpu_proxylib_http_kafka.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u bench.py --workload cfg2 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/cfg2.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --workload cfg2 --requests 50000000 --unique 1000000 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $O/cfg2_50m.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/cfg5.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/exp_mixed.py 8000000 > $O/mx.log 2>&1 || exit 5
python3 - <<PY
import json
for f in ("cfg2", "cfg2_50m", "cfg5"):
    for line in open(f"$O/{f}.log"):
        if line.startswith("{"):
            d = json.loads(line)
            print(f, d["ms_per_step"], {k: (v["ms"], v["frac"]) for k, v in d.get("kernels", {}).items()}, d["parity"]["bit_exact"])
PY
grep "ms/step" $O/mx.log
