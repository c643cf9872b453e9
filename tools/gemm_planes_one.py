"""Run one planes-GEMM shape repeatedly (rocprofv3 counter passes):
python tools/gemm_planes_one.py M N K a_rc b_rc reps"""
import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rl_ctr_prediction_amd import hip_ops as H  # noqa: E402
M, N, K, a_rc, b_rc, reps = (int(v) for v in sys.argv[1:7])
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(*((K, M) if a_rc else (M, K)), device="cuda", generator=g)
Bm = torch.randn(*((K, N) if b_rc else (N, K)), device="cuda", generator=g)
pa, pb = H.split_planes(A), H.split_planes(Bm)
out = torch.empty(M, N, device="cuda")
for _ in range(reps):
    H.gemm_planes(pa, pb, bool(a_rc), bool(b_rc), out=out)
torch.cuda.synchronize()
