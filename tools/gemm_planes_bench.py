"""Time the DeepFM MLP GEMMs (C3: B=8192, 1664-300-200) on pre-split planes, in the
orientations the fused trainer uses, per tiling / split-K (CTR_GEMM_PLANES_CFG).

    python tools/gemm_planes_bench.py [--reps 20] [--sweep] [--B 8192] [--W 1664]

Prints one JSON line per (shape, config): microseconds per launch (HIP events around
`reps` back-to-back launches, median of 3 groups), fp32-equivalent TFLOP/s (2*M*N*K) and
the bf16 MFMA rate actually issued (6 products).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rl_ctr_prediction_amd import hip_ops as H  # noqa: E402


def pg_shapes(n=4096):
    """The C4 policy MLP (741-1024-512-256 planes layers) at an episode of n transitions."""
    return {"pg fwd0 S.W0^T": (n, 1024, 741, False, False),
            "pg fwd1 H1.W1^T": (n, 512, 1024, False, False),
            "pg fwd2 H2.W2^T": (n, 256, 512, False, False),
            "pg d1 G2.W2": (n, 512, 256, False, True),
            "pg d0 G1.W1": (n, 1024, 512, False, True),
            "pg dW2 G2^T.H2": (256, 512, n, True, True),
            "pg dW1 G1^T.H1": (512, 1024, n, True, True),
            "pg dW0 G0^T.S": (1024, 741, n, True, True)}


def shapes(B, W, H1=300, H2=200):
    # name: (M, N, K, a_rc, b_rc)
    return {"fwd0 X.W0^T": (B, H1, W, False, False),
            "fwd1 H1.W1^T": (B, H2, H1, False, False),
            "dH1 dH2.W1": (B, H1, H2, False, True),
            "dX dH1.W0": (B, W, H1, False, True),
            "dW1 dH2^T.H1": (H2, H1, B, True, True),
            "dW0 dH1^T.X": (H1, W, B, True, True)}


def time_one(pa, pb, a_rc, b_rc, out, reps):
    H.gemm_planes(pa, pb, a_rc, b_rc, out=out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            H.gemm_planes(pa, pb, a_rc, b_rc, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(ts)[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--sweep", action="store_true", help="every tiling x split-K in {1,2,4,8}")
    ap.add_argument("--B", type=int, default=8192)
    ap.add_argument("--W", type=int, default=1664)
    ap.add_argument("--tiles", type=int, default=25, help="sweep tilings 0 .. tiles-1")
    ap.add_argument("--only", default="", help="comma-separated tiling indices to sweep")
    ap.add_argument("--pg", action="store_true", help="the C4 policy MLP shapes instead")
    ap.add_argument("--splits", default="1,2,4,8", help="split-K values of the sweep")
    ap.add_argument("--xg", default="1", help="XCD N-group values of the sweep (third cfg field)")
    ap.add_argument("--shapes", default="", help="comma-separated shape-name prefixes to run")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    total = 0.0
    table = pg_shapes() if args.pg else shapes(args.B, args.W)
    for name, (M, N, K, a_rc, b_rc) in table.items():
        if args.shapes and not any(name.startswith(p) for p in args.shapes.split(",")):
            continue
        A = torch.randn(*((K, M) if a_rc else (M, K)), device=dev, generator=g)
        Bm = torch.randn(*((K, N) if b_rc else (N, K)), device=dev, generator=g)
        pa, pb = H.split_planes(A), H.split_planes(Bm)
        out = torch.empty(M, N, device=dev)
        cfgs = ["auto"]
        if args.sweep:
            tiles = [int(t) for t in args.only.split(",")] if args.only else range(args.tiles)
            cfgs += [f"{t},{s},{x}" for t in tiles for s in map(int, args.splits.split(","))
                     for x in map(int, args.xg.split(","))
                     if not (b_rc and t in (0, 6, 8, 9))]
        best = None
        for cfg in cfgs:
            if cfg == "auto":
                os.environ.pop("CTR_GEMM_PLANES_CFG", None)
            else:
                os.environ["CTR_GEMM_PLANES_CFG"] = cfg
            chosen = H.gemm_planes_config(a_rc, b_rc, M, N, K)
            if cfg != "auto" and chosen["tile"] != int(cfg.split(",")[0]):
                continue  # not valid for this shape (the library fell back to its choice)
            us = time_one(pa, pb, a_rc, b_rc, out, args.reps)
            tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
            print(json.dumps({"shape": name, "cfg": cfg, "chosen": chosen, "us": round(us, 2),
                              "TFLOPs_fp32eq": round(tf, 1), "bf16_TFLOPs": round(6 * tf, 1)}),
                  flush=True)
            if cfg == "auto":
                auto_us = us
            if best is None or us < best[1]:
                best = (cfg, us)
        os.environ.pop("CTR_GEMM_PLANES_CFG", None)
        total += auto_us
        if args.sweep:
            print(json.dumps({"shape": name, "best": best[0], "us": round(best[1], 2)}), flush=True)
    print(json.dumps({"sum_auto_us": round(total, 1)}))


if __name__ == "__main__":
    main()
