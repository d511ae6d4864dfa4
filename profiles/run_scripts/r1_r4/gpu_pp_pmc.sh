#!/bin/bash
# PMC passes over one gemm_pp config and hipBLASLt on the same shape (each pass its own rocprofv3 run).
# Env: OP (gate_up), CFG (0), SK (1), M (1024)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OP=${OP:-gate_up}; CFG=${CFG:-0}; SK=${SK:-1}; M=${M:-1024}
out=gpurun_out/pmc_${OP}_${CFG}_${SK}
mkdir -p $out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVES TCC_HIT_sum TCC_MISS_sum"
for who in pp lib; do
  extra=""; [ $who = lib ] && extra="--lib"
  i=0
  for P in "$P1" "$P2"; do
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $out/${who}_p$i -o run -- \
      python3 scripts/pp_one.py --op $OP --m $M --cfg $CFG --sk $SK --iters 10 $extra > $out/${who}_p$i.log 2>&1 || exit $?
    i=$((i+1))
  done
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python3 scripts/pp_one.py --op $OP --m $M --cfg $CFG --sk $SK --iters 10 > $out/trace.log 2>&1 || exit $?
echo done
