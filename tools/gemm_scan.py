"""Time one tiling over K (fixed M, N) to split per-block fixed cost from the k-loop:
python tools/gemm_scan.py CFG M N ta tb K1,K2,..."""
import json, os, sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rl_ctr_prediction_amd import hip_ops as H  # noqa: E402
cfg, M, N, ta, tb, Ks = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
os.environ["CTR_GEMM_CFG"] = cfg
for K in (int(k) for k in Ks.split(",")):
    a = torch.randn(*((K, M) if ta else (M, K)), device="cuda")
    b = torch.randn(*((N, K) if tb else (K, N)), device="cuda")
    out = torch.empty(M, N, device="cuda")
    for _ in range(3):
        H.gemm(a, b, bool(ta), bool(tb), out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        H.gemm(a, b, bool(ta), bool(tb), out=out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(json.dumps({"cfg": cfg, "M": M, "N": N, "K": K, "us": round(us, 2),
                      "TF": round(2 * M * N * K / us / 1e6, 1)}), flush=True)
