# PMC passes over one command (GPU box): one rocprofv3 run per counter group
# (never more than the per-block limits; no trace domains combined with --pmc).
# usage: bash tools/pmc_run.sh OUTDIR cmd args...
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$1; shift
mkdir -p $out
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $out/pmc$i -o pmc --output-format csv -- "$@" > $out/log_$i.txt 2>&1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/stats -o stats --output-format csv -- "$@" > $out/log_stats.txt 2>&1
