#!/bin/bash
# GPU-box runner: each GPU step under its own time limit; stop at the first
# crash / abort / timeout (exit >= 124), continue past ordinary test failures.
# Usage: tools/gpu_check.sh <tag> [steps...]   steps: smoke tests bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -5 "$OUT/$name.log"
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
for step in "$@"; do
    case $step in
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    ktests) run ktests 400 python -u -m pytest tests/test_gpu_kafka.py tests/test_gpu_memcache.py tests/test_gpu_proxylib.py -m gpu -v --timeout 120 --timeout-method thread ;;
    mctests) run mctests 400 python -u -m pytest tests/test_gpu_memcache.py -m gpu -v --timeout 120 --timeout-method thread ;;
    tests) run tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    testsall) run testsall 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    bench) run bench 600 python -u bench.py ;;
    benchq) run benchq 400 python -u bench.py --steps 5 --warmup 2 ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o prof --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    pmc)
        i=0
        for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
                    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" \
                    "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_BUSY_max TCP_TCC_READ_REQ_sum"; do
            i=$((i+1))
            run pmc$i 180 rocprofv3 --pmc $ctrs -d "$OUT/pmc$i" -o pmc --output-format csv -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline
        done ;;
    bench_cfg*) run $step 900 python -u bench.py --workload ${step#bench_} --steps 10 --warmup 3 ;;
    prof_cfg*) run $step 900 rocprofv3 --kernel-trace --stats -d "$OUT/$step" -o prof --output-format csv -- python3 -u bench.py --workload ${step#prof_} --steps 10 --warmup 2 --no-cpu-baseline ;;
    pmc_cfg*)
        wl=${step#pmc_}; i=0
        for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
                    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" \
                    "FETCH_SIZE" "WRITE_SIZE"; do
            i=$((i+1))
            run ${step}_$i 180 rocprofv3 --pmc $ctrs -d "$OUT/${step}_$i" -o pmc --output-format csv -- python3 -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline
        done ;;
    fetch_cfg*) run $step 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/$step" -o pmc --output-format csv -- python3 -u bench.py --workload ${step#fetch_} --steps 3 --warmup 1 --no-cpu-baseline ;;
    write_cfg*) run $step 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/$step" -o pmc --output-format csv -- python3 -u bench.py --workload ${step#write_} --steps 3 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $step" ;;
    esac
done
