set -o pipefail
O=gpurun_out/mc2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/cfg5.log 2>&1 || exit 4
python3 - <<PY
import json
for line in open("$O/cfg5.log"):
    if line.startswith("{"):
        d = json.loads(line)
        print("cfg5", d["ms_per_step"], {k: (v["ms"], v["frac"]) for k, v in d.get("kernels", {}).items()}, d["parity"]["bit_exact"])
PY
