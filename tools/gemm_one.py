"""Run one GEMM shape repeatedly (for rocprofv3 counter passes): python tools/gemm_one.py M N K ta tb reps"""
import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rl_ctr_prediction_amd import hip_ops as H  # noqa: E402
M, N, K, ta, tb, reps = (int(v) for v in sys.argv[1:7])
g = torch.Generator(device="cuda").manual_seed(0)
a = torch.randn(*((K, M) if ta else (M, K)), device="cuda", generator=g)
b = torch.randn(*((N, K) if tb else (K, N)), device="cuda", generator=g)
out = torch.empty(M, N, device="cuda")
for _ in range(reps):
    H.gemm(a, b, bool(ta), bool(tb), out=out)
torch.cuda.synchronize()
