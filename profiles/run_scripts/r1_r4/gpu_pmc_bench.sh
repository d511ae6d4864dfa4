#!/bin/bash
# PMC passes over one headline wave (kernel counters only, one group per run): per-kernel VALU / MFMA / LDS
# instruction counts and wave cycles, to find issue-bound kernels.  Usage (gpurun): bash scripts/gpu_pmc_bench.sh
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcb
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY"
timeout -s KILL 400 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d /tmp/pmcb -o pmc -- \
    python3 bench.py --steps 1 --warmup 0 --single-stream 1 > gpurun_out/pmcb/p1.log 2>&1
rc=$?; echo "pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY' > gpurun_out/pmcb/summary.txt
import csv, glob, collections
f = glob.glob("/tmp/pmcb/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    n = r.get("Kernel_Name", "")
    n = n.replace("void ", "").split("(")[0][:60]
    agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[n].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
print(f"{'kernel':60s} {'disp':>6s} {'waveCyc':>10s} {'VALU/MFMA':>9s} {'VALU':>10s} {'MFMA':>9s} {'LDS':>9s} {'actVALU%':>8s} {'waitInst%':>9s}")
for n, c in rows[:30]:
    w = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{n:60s} {len(disp[n]):6d} {w:10.3g} {c['SQ_INSTS_VALU'] / max(1, c['SQ_INSTS_MFMA']):9.1f} {c['SQ_INSTS_VALU']:10.3g} "
          f"{c['SQ_INSTS_MFMA']:9.3g} {c['SQ_INSTS_LDS']:9.3g} {100 * c['SQ_ACTIVE_INST_VALU'] / w:8.1f} {100 * c['SQ_WAIT_INST_ANY'] / w:9.1f}")
PY
cat gpurun_out/pmcb/summary.txt
rm -rf /tmp/pmcb
