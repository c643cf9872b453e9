"""Reference point only (not a product path): hipBLASLt bf16 GEMM rate via torch.matmul on
the C3 MLP shapes with K' = 6K (the six plane products as one bf16 GEMM), to size the
headroom of the hand-written planes GEMM.  python tools/blas_ref.py"""
import json
import torch

dev = torch.device("cuda:0")
shapes = {"fwd0": (8192, 320, 1664), "dX": (8192, 1664, 320), "dW0": (320, 1664, 8192),
          "fwd1": (8192, 208, 320)}
for name, (M, N, K) in shapes.items():
    for kmul in (1, 6):
        a = torch.randn(M, K * kmul, device=dev).bfloat16()
        b = torch.randn(K * kmul, N, device=dev).bfloat16()
        for outf in ("bf16", "f32"):
            try:
                f = (lambda: torch.matmul(a, b)) if outf == "bf16" else \
                    (lambda: torch.mm(a, b, out_dtype=torch.float32))
                f()
            except Exception as e:  # out_dtype not supported
                print(json.dumps({"shape": name, "kmul": kmul, "out": outf, "error": str(e)[:80]}))
                continue
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    f()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 20)
            us = sorted(ts)[1]
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K * kmul, "out": outf,
                              "us": round(us, 2),
                              "bf16_TF": round(2 * M * N * K * kmul / us / 1e6, 1)}), flush=True)
