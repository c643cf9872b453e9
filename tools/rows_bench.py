"""Time the deferred-Adam catch-up of a batch's unique rows (deferred_rows_vec, what runs
ahead of the forward) at a config's shape, every row `--stale` steps behind:

    python tools/rows_bench.py [--config c3] [--stale 1,4,16,32] [--reps 20]

Prints one JSON line per staleness: us per launch (median), rows, replayed element-steps/s.
A/B against a tuning build with CTR_HIP_LIB (tools/build_variant.py).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--stale", default="1,4,16,32")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import bench
    from rl_ctr_prediction_amd import hip_ops as H
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    cfg = bench.CONFIGS[a.config]
    V, F, K, B = cfg["V"], cfg["F"], cfg["K"], cfg["B"]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    E = torch.randn(V, K, device=dev, generator=g).mul_(0.05)
    mE = torch.randn(V, K, device=dev, generator=g).mul_(1e-4)
    vE = torch.rand(V, K, device=dev, generator=g).mul_(1e-8)
    lin = torch.randn(V, device=dev, generator=g).mul_(0.05)
    ml, vl = torch.zeros_like(lin), torch.zeros_like(lin)
    last = torch.zeros(V, dtype=torch.int32, device=dev)
    x = torch.from_numpy(next(CriteoSynth(V, F, seed=1).batches(1, B))[0]).to(dev)
    P = H.SparsePlanBuffers(B * F, dev)
    P.build(x, V)
    U = P.num_unique_host()
    rows = P.unique_rows[:U].long()
    tab = H.AdamStepTable(1e-3, (0.9, 0.999), dev)
    step = 200
    for T in map(int, a.stale.split(",")):
        ts = []
        for r in range(a.reps + 2):
            last[rows] = step - T
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            H.adam_deferred_rows(E, mE, vE, lin, ml, vl, last, P, step, tab, weight_decay=1e-5)
            e1.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3)
        us = sorted(ts)[len(ts) // 2]
        print(json.dumps({"config": a.config, "stale": T, "rows": U, "us": us,
                          "elem_steps_per_s": U * (K + 1) * T / (us * 1e-6)}), flush=True)


if __name__ == "__main__":
    main()
