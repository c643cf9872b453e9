"""Run the six C3 MLP GEMM shapes on pre-split planes, REPS launches each, in a fixed order
(for rocprofv3 --pmc passes: tools/gemm_planes_pmc.sh), or summarise such passes:

    python tools/gemm_planes_pmc.py run [REPS]
    python tools/gemm_planes_pmc.py summary DIR [REPS]   (per-shape averages per counter)
"""
import collections
import csv
import glob
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
SHAPES = [("fwd0", 8192, 300, 1664, 0, 0), ("fwd1", 8192, 200, 300, 0, 0),
          ("dH1", 8192, 300, 200, 0, 1), ("dX", 8192, 1664, 300, 0, 1),
          ("dW1", 200, 300, 8192, 1, 1), ("dW0", 300, 1664, 8192, 1, 1)]


def run(reps):
    import torch
    from rl_ctr_prediction_amd import hip_ops as H
    g = torch.Generator(device="cuda").manual_seed(0)
    for _, M, N, K, a_rc, b_rc in SHAPES:
        A = torch.randn(*((K, M) if a_rc else (M, K)), device="cuda", generator=g)
        Bm = torch.randn(*((K, N) if b_rc else (N, K)), device="cuda", generator=g)
        pa, pb = H.split_planes(A), H.split_planes(Bm)
        out = torch.empty(M, N, device="cuda")
        torch.cuda.synchronize()
        for _ in range(reps):
            H.gemm_planes(pa, pb, bool(a_rc), bool(b_rc), out=out)
        torch.cuda.synchronize()


def summary(root, reps):
    vals = collections.defaultdict(list)  # (shape, counter) -> values
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if "gemm_planes_kernel" in r["Kernel_Name"]]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        order = {d: i for i, d in enumerate(ids)}
        for r in rows:
            shape = SHAPES[order[int(r["Dispatch_Id"])] // reps][0]
            vals[(shape, r["Counter_Name"])].append(float(r["Counter_Value"]))
    counters = sorted({c for _, c in vals})
    print("counter".ljust(28) + "".join(s[0].rjust(16) for s in SHAPES))
    for c in counters:
        print(c.ljust(28) + "".join(
            f"{sum(vals[(s[0], c)]) / max(len(vals[(s[0], c)]), 1):16.0f}" for s in SHAPES))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 10)
    else:
        summary(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 10)
