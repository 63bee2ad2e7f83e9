# Round-5 final measurement (GPU box), part 3: PMC groups of the kernels cfg5
# does not run -- cfg4's grouping kernels, the stream framers, the latency path.
set -o pipefail
O=gpurun_out/${TAG:-p6}; mkdir -p $O; export TMPDIR=/tmp
bash tools/pmc_run.sh $O/cfg4 python3 -u bench.py --workload cfg4 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-latency --no-streams --profile-steps 0 || exit 5
echo cfg4 done
bash tools/pmc_run.sh $O/frame_http python3 -u tools/exp_frame.py http 1000000 16384 || exit 6
bash tools/pmc_run.sh $O/frame_mc python3 -u tools/exp_frame.py memcache 1000000 16384 || exit 7
echo frame done
bash tools/pmc_run.sh $O/lat python3 -u tools/exp_lat.py || exit 8
echo lat done
