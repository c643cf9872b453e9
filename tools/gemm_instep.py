"""Median in-step duration of every planes-GEMM / reduce launch kind per variant traced by
tools/gemm_instep.sh:  python tools/gemm_instep.py gpurun_out/instep_*"""
import csv
import glob
import statistics
import sys

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not f:
        continue
    agg = {}
    for r in csv.DictReader(open(f[0])):
        n = r["Kernel_Name"]
        if "gemm_planes_kernel" not in n and "planes_reduce" not in n:
            continue
        key = (n.split("(")[0].replace("void ctr::", "")[:60], int(r["Grid_Size_X"]) // 64)
        agg.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(d)
    for (name, waves), v in sorted(agg.items(), key=lambda kv: -statistics.median(kv[1])):
        print(f"   {name:60s} waves={waves:6d} n={len(v):4d} median={statistics.median(v):7.1f} us")
