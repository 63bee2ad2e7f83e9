# Diagnosis (GPU box): HTTP phase split (timing build) on cfg5's HTTP requests,
# then the PMC passes of tools/pmc_run.sh over one cfg5 step.
# usage: TAG=x [PMC=1] bash tools/run_diag.sh
set -o pipefail
O=gpurun_out/${TAG:-diag}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/exp_phase.py 4000000 > $O/phase_product.log 2>&1 || { tail -20 $O/phase_product.log; exit 1; }
cat $O/phase_product.log | grep -v amdgpu.ids
EXP_LIB=libl7gpu_timing.so timeout -k 10 300 python3 -u tools/exp_phase.py 4000000 > $O/phase_timing.log 2>&1 || { tail -20 $O/phase_timing.log; exit 2; }
cat $O/phase_timing.log | grep -v amdgpu.ids
if [ "${PMC:-1}" = 1 ]; then
  bash tools/pmc_run.sh $O/pmc python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-latency --profile-steps 0 || exit 3
  for k in http_classify kafka_classify memcache_classify; do echo "== $k"; python3 tools/pmc_summary.py $O/pmc $k 2>&1 | tail -30; done
fi
echo done
