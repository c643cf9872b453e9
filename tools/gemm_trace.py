"""Per-block timing of one GEMM launch (tuning build with -DCTR_GEMM_TRACE=1):

    CTR_HIP_LIB=rl_ctr_prediction_amd/variants/lib_trace.so \\
        python tools/gemm_trace.py M N K ta tb [cfg]

Prints the launch time (HIP events), the spread of block start times, and per block the
k-loop and epilogue cycles against the MFMA-only cycle count of its tile, split by XCD.
"""
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rl_ctr_prediction_amd import hip_ops as H  # noqa: E402
from rl_ctr_prediction_amd._lib import lib  # noqa: E402

M, N, K, ta, tb = (int(v) for v in sys.argv[1:6])
if len(sys.argv) > 6:
    os.environ["CTR_GEMM_CFG"] = sys.argv[6]
a = torch.randn(*((K, M) if ta else (M, K)), device="cuda")
b = torch.randn(*((N, K) if tb else (K, N)), device="cuda")
out = torch.empty(M, N, device="cuda")
for _ in range(5):
    H.gemm(a, b, bool(ta), bool(tb), out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
H.gemm(a, b, bool(ta), bool(tb), out=out)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3
dll = lib.load()
n = 16384
buf = (ctypes.c_ulonglong * (5 * n))()
dll.ctr_debug_gemm_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
dll.ctr_debug_gemm_trace(ctypes.addressof(buf), n)
t = np.frombuffer(buf, dtype=np.uint64).reshape(n, 5).astype(np.int64)
t = t[t[:, 0] > 0]
rt = (t[:, 0] - t[:, 0].min()) / 100.0  # s_memrealtime: 100 MHz -> us
loop = t[:, 2] - t[:, 1]
epi = t[:, 3] - t[:, 2]
xcc = t[:, 4] >> 8
q = lambda v: {"min": int(v.min()), "p50": int(np.median(v)), "max": int(v.max())}  # noqa: E731
res = {"M": M, "N": N, "K": K, "cfg": os.environ.get("CTR_GEMM_CFG", "auto"), "us": round(us, 1),
       "TF": round(2 * M * N * K / us / 1e6, 1), "blocks": len(t),
       "start_spread_us": round(float(rt.max()), 2), "start_p50_us": round(float(np.median(rt)), 2),
       "loop_cycles": q(loop), "epilogue_cycles": q(epi),
       "per_xcc_loop_p50": {int(x): int(np.median(loop[xcc == x])) for x in np.unique(xcc)},
       "per_xcc_blocks": {int(x): int((xcc == x).sum()) for x in np.unique(xcc)}}
print(json.dumps(res), flush=True)
