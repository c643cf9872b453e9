"""Per-kernel summary of tools/scatter_pmc.sh: for every run (alone_c3, alone_c5, step_c3)
and every scatter kernel (seg_chunk / seg_combine*), the average kernel duration from the
trace and the counters of the PMC passes, with the derived figures:

  wait_frac   SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barrier)
  issue_frac  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  active_frac SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  waves_cu    SQ_LEVEL_WAVES / SQ_BUSY_CYCLES / 256 CUs (mean waves resident per CU)
  l2_hit      TCC_HIT / (TCC_HIT + TCC_MISS)
  hbm_MB      FETCH_SIZE x 2 (gfx950: wide reads tallied at half) + WRITE_SIZE, in MB
  GBps        hbm bytes / average duration

    python tools/scatter_pmc_summary.py gpurun_out/scatter_pmc [--json out.json]
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import sys

KERNELS = ("seg_chunk_kernel", "seg_combine_apply_kernel", "seg_combine_kernel")


def short(name: str) -> str | None:
    for k in KERNELS:
        if k in name:
            return k
    return None


def main():
    root = sys.argv[1]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    dur = collections.defaultdict(list)
    ctr = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "*_trace", "**", "*kernel_trace.csv"), recursive=True):
        run = os.path.relpath(f, root).split(os.sep)[0][: -len("_trace")]
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                dur[(run, k)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for f in glob.glob(os.path.join(root, "*_p[0-9]", "**", "*counter_collection.csv"),
                       recursive=True):
        run = os.path.relpath(f, root).split(os.sep)[0].rsplit("_p", 1)[0]
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                ctr[(run, k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    res = {}
    for (run, k), d in sorted(dur.items()):
        c = {n: sum(v) / len(v) for (r2, k2, n), v in ctr.items() if r2 == run and k2 == k}
        e = {"n": len(d), "us_avg": sum(d) / len(d), "us_min": min(d)}
        e.update({n: c[n] for n in sorted(c)})
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for a, b in (("wait_frac", "SQ_WAIT_ANY"), ("issue_frac", "SQ_WAIT_INST_ANY"),
                         ("active_frac", "SQ_ACTIVE_INST_ANY")):
                if b in c:
                    e[a] = c[b] / wc
        if c.get("SQ_BUSY_CYCLES") and "SQ_LEVEL_WAVES" in c:
            e["waves_cu"] = c["SQ_LEVEL_WAVES"] / c["SQ_BUSY_CYCLES"] / 256
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            e["l2_hit"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            mb = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024 / 1e6  # counters are in KiB
            e["hbm_MB"] = mb
            e["GBps"] = mb * 1e6 / (e["us_avg"] * 1e-6) / 1e9
        res[f"{run}/{k}"] = e
        keys = ("us_avg", "us_min", "wait_frac", "issue_frac", "active_frac", "waves_cu",
                "l2_hit", "hbm_MB", "GBps")
        print(f"{run:10s} {k:26s} " + " ".join(
            f"{x}={e[x]:.3f}" for x in keys if x in e), flush=True)
    if out_json:
        json.dump(res, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main()
