#!/bin/bash
# PMC passes (each counter set its own rocprofv3 run) over gemm_lg configs and hipBLASLt at 8192^3.
# CFGS env: space-separated config ids, "lib" for hipBLASLt
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFGS=${CFGS:-"20 65 lib"}
out=gpurun_out/lgpmc
mkdir -p $out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVES TCC_HIT_sum TCC_MISS_sum"
P3="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum"
for c in $CFGS; do
  if [ $c = lib ]; then arg="--cfg 0 --lib"; else arg="--cfg $c"; fi
  i=0
  for P in "$P1" "$P2" "$P3"; do
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $out/c${c}_p$i -o run -- \
      python3 scripts/pp_one.py --op sq --m 8192 $arg --sk 1 --iters 6 > $out/c${c}_p$i.log 2>&1 || { echo "c$c p$i rc=$?"; tail -5 $out/c${c}_p$i.log; exit 1; }
    i=$((i+1))
  done
done
python3 scripts/pmc_table.py $out > $out/table.txt 2>&1
find $out -name "*.csv" -size +2M -delete
cat $out/table.txt
