# Round-6 final measurement (GPU box), part 2: FETCH_SIZE / WRITE_SIZE passes
# per workload (profiles/traffic_<wl>.json via tools/traffic.py) and the PMC
# groups (tools/pmc_run.sh) of one cfg5 step.   usage: TAG=p bash tools/run_r6_pmc.sh
set -o pipefail
O=gpurun_out/${TAG:-p}; mkdir -p $O; export TMPDIR=/tmp
for wl in ${WLS:-cfg2 cfg3 cfg5}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c -d $O/${wl}_$c -o pmc --output-format csv -- python3 -u bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-latency --no-streams --profile-steps 0 > $O/${wl}_$c.log 2>&1 || exit 4
  done
  echo traffic $wl
done
if [ "${GROUPS_ON:-1}" = 1 ]; then
  bash tools/pmc_run.sh $O/groups python3 -u bench.py --workload ${PMC_WL:-cfg5} --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-latency --no-streams --profile-steps 0 || exit 5
  echo groups done
fi
