# TA / TCP PMC passes (GPU box) over one cfg5 step: is a kernel bound by the
# vector-memory address path (TA busy, L1->L2 latency)?
# usage: bash tools/pmc_ta.sh OUTDIR
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$1; mkdir -p $out
i=0
for ctrs in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
            "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctrs -d $out/pmc$i -o pmc --output-format csv -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-latency --profile-steps 0 > $out/log_$i.txt 2>&1
done
for k in http_classify kafka_classify memcache_classify; do echo "== $k"; python3 tools/pmc_summary.py $out $k; done
