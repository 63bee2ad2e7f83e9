# Evidence passes for the shipped build (GPU box): FETCH/WRITE traffic per
# workload (tools/run_traffic.sh) and the SQ/TA/TCP counter sets over one cfg5
# step (tools/pmc_run.sh, tools/pmc_ta.sh).  usage: TAG=x bash tools/run_evidence.sh
set -o pipefail
O=gpurun_out/${TAG:-ev}; mkdir -p $O
WLS="${WLS:-cfg5 cfg2 cfg3}" bash tools/run_traffic.sh || exit 1
bash tools/pmc_run.sh $O/pmc python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-latency --profile-steps 0 || exit 2
bash tools/pmc_ta.sh $O/pmcta > $O/pmcta.txt 2>&1 || exit 3
for k in http_classify kafka_classify memcache_classify partition_kernel; do echo "== $k"; python3 tools/pmc_summary.py $O/pmc $k; done > $O/pmc_summary.txt
echo done
