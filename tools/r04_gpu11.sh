#!/bin/bash
# IPNN backward: timing of the kernels and counters of the default one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ipnn_bwd_bench.py > gpurun_out/r04_ipnn_bwd.txt 2>&1 || { cat gpurun_out/r04_ipnn_bwd.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_ipnn_bwd.txt
OUT=gpurun_out/ipnn_pmc; rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d $OUT -o run -- \
  python3 tools/ipnn_bwd_bench.py --kernels default --reps 3 > $OUT/run.log 2>&1 || { tail -5 $OUT/run.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/ipnn_pmc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "ipnn_backward" in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: sum(v) / len(v) for c, v in d.items()})
PY
