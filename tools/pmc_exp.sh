set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r1h
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" \
            "FETCH_SIZE" "TA_BUSY_avr TA_BUSY_max TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  for v in c e; do
    timeout -k 10 120 rocprofv3 --pmc $ctrs -d gpurun_out/r1h/pmc${i}_$v -o pmc --output-format csv -- python3 -u tools/exp_http.py 1000000 $v > gpurun_out/r1h/log_${i}_$v.txt 2>&1
  done
done
