#!/bin/bash
# r5: flash prefill (attn_prefill2, fp8 KV, 16k chunk over a 112k prefix): timing, then two PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=${PMC_OUT:-gpurun_out/r5ppmc}
export PMC_OUT=$O
mkdir -p $O
timeout -k 10 200 python -u scripts/bench_prefill_attn.py --variants 2 --cases chunk16k_prefix112k,chunk16k_prefix0 > $O/t_bf16.log 2>&1 || { tail -20 $O/t_bf16.log; exit 1; }
grep '^{' $O/t_bf16.log
timeout -k 10 200 python -u scripts/bench_prefill_attn.py --variants 2 --fp8 --cases chunk16k_prefix112k > $O/t_fp8.log 2>&1 || { tail -20 $O/t_fp8.log; exit 1; }
grep '^{' $O/t_fp8.log
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA"
P2="SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o pmc -- python3 scripts/bench_prefill_attn.py --variants 2 --fp8 --cases chunk16k_prefix112k > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob(""+__import__("os").environ.get("PMC_OUT","gpurun_out/r5ppmc")+"/p*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "attn_prefill" not in r.get("Kernel_Name", ""):
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    for k in sorted(agg):
        print(f"  {k:28s} {agg[k] / max(1, n[k]):.4g} per dispatch-record ({n[k]} records)")
PY
find $O -name "*.csv" -size +2M -delete
