# cfg2 at 1M vs tiled 50M requests: does the per-request HTTP time depend on the arena size? (GPU box)
set -o pipefail
O=gpurun_out/tlb; mkdir -p $O
for r in 1000000 20000000 50000000; do
  timeout -k 10 300 python -u bench.py --workload cfg2 --requests $r --unique 1000000 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $O/cfg2_$r.log 2>&1 || exit 1
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/tlb/cfg2_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            k = d["kernels"]["http"]
            print(f, d["config"]["requests_per_gpu"], "http ms", k["ms"], "ns/req", 1e6 * k["ms"] / d["config"]["requests_per_gpu"], "frac", k["frac"])
PY
