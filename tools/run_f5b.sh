set -o pipefail
# framing tests + throughput, then a cfg5 bench line with the streams leg
O=gpurun_out/f5b; mkdir -p $O
bash tools/run_f5.sh > $O/f5.log 2>&1 || { tail -30 $O/f5.log; exit 1; }
grep -v "amdgpu.ids" $O/f5.log | grep -v "kafka:\|classify (host"
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-latency > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], d['roofline']['frac'], json.dumps(d['streams']), json.dumps(d['kernels']))"
