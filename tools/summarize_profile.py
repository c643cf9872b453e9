"""Summarise a rocprofv3 run (tools/gpu_profile.sh output) into profiles/:
<tag>_<cfg>_kernel_stats.csv (copied) and <tag>_pmc.json (HBM bytes per launch per kernel,
FETCH_SIZE x2 for gfx950 wide streaming reads (MI355X_MICROARCH.md §HBM), WRITE_SIZE as-is;
both counters are in KiB)."""
import collections, csv, json, shutil, sys
from pathlib import Path

tag = sys.argv[1]
cfgs = sys.argv[2:] or ["c3", "c2"]
root = Path(__file__).resolve().parents[1]
out = {}
pmc_path = root / "profiles" / f"{tag}_pmc.json"
if pmc_path.exists():
    out = json.loads(pmc_path.read_text())
for cfg in cfgs:
    base = root / "gpurun_out" / f"prof_{tag}_{cfg}"
    shutil.copy(base / "trace" / "run_kernel_stats.csv", root / "profiles" / f"{tag}_{cfg}_kernel_stats.csv")
    vals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(base / f"pmc_{c}" / "run_counter_collection.csv")):
            name = r["Kernel_Name"]
            short = name.split("(")[0].replace("void ", "").split("::")[-1].split("<")[0]
            agg[short].append(float(r["Counter_Value"]))
        # all MLP GEMM launches together (gemm_sb16_kernel + gemm_f32_kernel): the unit
        # bench.py's GEMM roofline averages over
        g = [x for k, v in agg.items() if k.startswith("gemm_") for x in v]
        if g:
            agg["gemm"] = g
        vals[c] = {k: sum(v) / len(v) for k, v in agg.items()}
    kern = {}
    for k in vals["FETCH_SIZE"]:
        if k not in vals["WRITE_SIZE"]:
            continue
        f, w = vals["FETCH_SIZE"][k] * 1024 * 2, vals["WRITE_SIZE"][k] * 1024
        kern[k] = {"fetch_bytes_per_launch": f, "write_bytes_per_launch": w,
                   "hbm_bytes_per_launch": f + w,
                   "note": "FETCH_SIZE(KiB)*1024*2 (gfx950 correction) + WRITE_SIZE(KiB)*1024"}
    out[cfg] = kern
pmc_path.write_text(json.dumps(out, indent=1))
print(json.dumps({c: {k: round(v["hbm_bytes_per_launch"] / 1e9, 4) for k, v in d.items()
                      if v["hbm_bytes_per_launch"] > 1e7} for c, d in out.items()}, indent=1))
