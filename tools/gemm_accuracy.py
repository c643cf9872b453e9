"""Error of both GEMM algorithms against an fp64 product, relative to the L1 bound
|A|.|B| (max and mean over the output), on the DeepFM / PG MLP shapes.

    python tools/gemm_accuracy.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rl_ctr_prediction_amd import hip_ops as H  # noqa: E402

SHAPES = [(8192, 300, 1664, False, True), (300, 1664, 8192, True, False),
          (8192, 1664, 300, False, False), (8192, 200, 300, False, True),
          (4096, 1024, 741, False, True), (1024, 741, 4096, True, False)]


def main():
    g = torch.Generator().manual_seed(5)
    for (M, N, K, ta, tb) in SHAPES:
        A = torch.randn(M, K, generator=g) * 0.1
        Bm = torch.randn(K, N, generator=g)
        a = (A.t() if ta else A).contiguous().cuda()
        b = (Bm.t() if tb else Bm).contiguous().cuda()
        ref = A.double() @ Bm.double()
        bound = A.double().abs() @ Bm.double().abs()
        row = {"shape": [M, N, K, ta, tb]}
        for name, algo in (("exact", H.GEMM_EXACT_F32), ("split", H.GEMM_SPLIT_BF16)):
            C = H.gemm(a, b, ta, tb, algo=algo).cpu().double()
            r = (C - ref).abs() / bound
            row[name] = {"max": float(r.max()), "mean": float(r.mean())}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
