# Kafka single-list partition + XCD mapping: tests, cfg3/cfg5 benches, cfg5 PMC per kernel (GPU box)
set -o pipefail
O=gpurun_out/${TAG:-k2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kafka.py tests/test_gpu_kafka_compressed.py tests/test_gpu_unowned.py tests/test_gpu_cfg4.py tests/test_gpu_memcache.py tests/test_gpu_proxylib_http_kafka.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u bench.py --workload cfg3 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/cfg3.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/cfg5.log 2>&1 || exit 3
python3 - <<PY
import json
for f in ("cfg3", "cfg5"):
    for line in open(f"$O/{f}.log"):
        if line.startswith("{"):
            d = json.loads(line)
            print(f, d["ms_per_step"], {k: (v["ms"], v["frac"]) for k, v in d.get("kernels", {}).items()}, d["parity"]["bit_exact"])
PY
if [ -n "$PMC" ]; then
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $c -d $O/pmc_$n -o pmc --output-format csv -- python3 -u bench.py --workload ${PMCWL:-cfg3} --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --profile-steps 0 > $O/pmc_$n.log 2>&1 || exit 4
done
fi
