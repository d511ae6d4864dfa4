#!/bin/bash
# PMC passes (each counter set its own rocprofv3 run) over gemm_lg configs at 8192^3: CFGS env (space-separated)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFGS=${CFGS:-"20 54 65"}
out=gpurun_out/lgpmc
mkdir -p $out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVES SQ_INST_CYCLES_VMEM SQ_LDS_ADDR_CONFLICT TA_BUSY_avr TA_TA_BUSY_sum"
for c in $CFGS; do
  i=0
  for P in "$P1" "$P2"; do
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $out/c${c}_p$i -o run -- \
      python3 scripts/pp_one.py --op sq --m 8192 --cfg $c --sk 1 --iters 6 > $out/c${c}_p$i.log 2>&1 || exit $?
    i=$((i+1))
  done
done
python3 scripts/pmc_table.py $out > $out/table.txt 2>&1
cat $out/table.txt
