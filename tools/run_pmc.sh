# PMC passes for one bench workload (GPU box): WL=cfg5 TAG=name bash tools/run_pmc.sh
set -o pipefail
O=gpurun_out/${TAG:-pmc}; mkdir -p $O
export TMPDIR=/tmp
WL=${WL:-cfg5}
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 170 rocprofv3 --pmc $c -d $O/pmc_$n -o pmc --output-format csv -- python3 -u bench.py --workload $WL --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --profile-steps 0 ${BENCHARGS:-} > $O/pmc_$n.log 2>&1 || exit 4
done
