# A/B bench lines + partition traffic of the product (GPU box)
set -o pipefail
O=gpurun_out/${TAG:-abt}; mkdir -p $O; export TMPDIR=/tmp
VARS="${VARS:-}" WLS="${WLS:-cfg5}" TAG=${TAG:-abt} bash tools/run_ab3.sh || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 170 rocprofv3 --pmc $c -d $O/cfg5_$c -o pmc --output-format csv -- python3 -u bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-latency --profile-steps 0 > $O/cfg5_$c.log 2>&1 || exit 6
done
echo traffic done
