set -o pipefail
mkdir -p gpurun_out/h1
timeout -k 10 300 python -u -m pytest tests/test_gpu_http.py tests/test_gpu_nfa.py tests/test_gpu_cfg4.py tests/test_gpu_unowned.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/h1/t.log 2>&1 || { tail -30 gpurun_out/h1/t.log; exit 1; }
tail -3 gpurun_out/h1/t.log
timeout -k 10 300 python -u bench.py --workload cfg2 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/h1/cfg2.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/h1/cfg5.log 2>&1 || exit 3
python3 - <<'PY'
import json
for f in ("cfg2", "cfg5"):
    for line in open(f"gpurun_out/h1/{f}.log"):
        if line.startswith("{"):
            d = json.loads(line)
            print(f, d["ms_per_step"], {k: (v["ms"], v["frac"]) for k, v in d.get("kernels", {}).items()}, d["parity"])
PY
