# FETCH_SIZE / WRITE_SIZE passes per workload (GPU box): WLS="cfg2 cfg3 cfg5" bash tools/run_traffic.sh
set -o pipefail
O=gpurun_out/traffic; mkdir -p $O; export TMPDIR=/tmp
for wl in ${WLS:-cfg2 cfg3 cfg5}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 170 rocprofv3 --pmc $c -d $O/${wl}_$c -o pmc --output-format csv -- python3 -u bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --profile-steps 0 > $O/${wl}_$c.log 2>&1 || exit 4
  done
done
echo done
