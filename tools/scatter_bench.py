"""Time the embedding scatter (segmented row sums) at a config's batch shape, in variants
that isolate its inputs: FM + dX (the DeepFM step), FM only (no dX), and the generic
segmented sum of a [S, K] value array (MODE_VALS).

    python tools/scatter_bench.py [--config c3|c2|c5] [--reps 50]

Run under rocprofv3 --kernel-trace --stats for the per-kernel split (chunk vs combine).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rl_ctr_prediction_amd import hip_ops as H  # noqa: E402
from rl_ctr_prediction_amd.synthetic import CriteoSynth  # noqa: E402

CONFIGS = {"c2": (1_000_000, 16, 4096, 26), "c3": (10_000_000, 64, 8192, 26),
           "c5": (40_000_000, 128, 8192, 22)}


def timed(fn, reps):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--uniform", action="store_true")
    args = ap.parse_args()
    V, K, B, F = CONFIGS[args.config]
    dev = torch.device("cuda:0")
    gen = CriteoSynth(V, F, uniform=args.uniform)
    import numpy as np
    x = torch.tensor(gen.ids(np.random.default_rng(1), B), device=dev)
    S = B * F
    plan = H.SparsePlanBuffers(S, dev).build(x, V)
    torch.cuda.synchronize()
    U = plan.num_unique_host()
    g = torch.Generator(device=dev).manual_seed(0)
    E = torch.randn(V, K, device=dev, generator=g) * 0.01
    gz = torch.randn(B, device=dev, generator=g)
    sum_e = torch.randn(B, K, device=dev, generator=g)
    dx = torch.randn(S, K, device=dev, generator=g)
    rows, lin = torch.empty(S, K, device=dev), torch.empty(S, device=dev)
    res = {"config": args.config, "S": S, "U": U}
    res["plan_us"] = timed(lambda: plan.build(x, V), args.reps)
    res["fm_dx_us"] = timed(lambda: H.fm_embedding_grad(plan, F, E, gz, sum_e, dx,
                                                        grad_rows=rows, grad_lin=lin), args.reps)
    res["fm_only_us"] = timed(lambda: H.fm_embedding_grad(plan, F, E, gz, sum_e, None,
                                                          grad_rows=rows, grad_lin=lin), args.reps)
    res["vals_us"] = timed(lambda: H.segment_sum_rows(plan, dx, out=rows), args.reps)
    # the fused path of the step: sums + the deferred Adam apply of the batch's rows
    table = (E, torch.zeros_like(E), torch.zeros_like(E), torch.zeros(V, device=dev),
             torch.zeros(V, device=dev), torch.zeros(V, device=dev),
             torch.zeros(V, dtype=torch.int32, device=dev))
    st = H.AdamStepTable(1e-3, (0.9, 0.999), dev)
    step_dev = torch.ones(1, dtype=torch.int32, device=dev)
    res["fm_dx_adam_us"] = timed(lambda: H.fm_embedding_grad_adam(
        plan, F, gz, sum_e, dx, table, step_dev, st, 1, weight_decay=1e-5, grad_rows=rows,
        grad_lin=lin), args.reps)
    # algorithmic bytes of the FM + dX scatter: per slot 4 index arrays (16 B) + dX row;
    # per unique row the table row read + the gradient row written (+ lin)
    alg = S * (16 + 4 * K) + U * (8 * K + 8) + B * 4 * K
    res["fm_dx_alg_bytes"] = alg
    res["fm_dx_GBps"] = alg / (res["fm_dx_us"] * 1e-6) / 1e9
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
