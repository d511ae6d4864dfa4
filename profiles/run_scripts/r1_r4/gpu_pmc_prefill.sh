#!/bin/bash
# PMC passes (kernel trace + counters only, one counter group per run) over the flash prefill kernel on the 48k-prefix
# chunk.  Usage (gpurun): bash scripts/gpu_pmc_prefill.sh [variant]
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
V=${1:-2}
mkdir -p gpurun_out/pmc
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA"
P2="SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc/p$i -o pmc -- \
      python3 scripts/bench_prefill_attn.py --variants $V --cases chunk16k_prefix48k > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc/p*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "attn_prefill" not in r.get("Kernel_Name", ""):
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f)
    for k in sorted(agg):
        print(f"  {k:28s} {agg[k] / max(1, n[k]):.4g} per dispatch-record ({n[k]} records)")
PY
find gpurun_out/pmc -name "*.csv" -size +2M -delete
