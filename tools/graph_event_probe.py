"""Probe: do timing events recorded inside a captured HIP graph give kernel durations?"""
import torch
x = torch.randn(64 << 20, device="cuda")
y = torch.empty_like(x)
s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(3):
    y.copy_(x)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    y.mul_(2.0)
    s0.record()
    y.copy_(x)
    e0.record()
    y.add_(1.0)
torch.cuda.synchronize()
for i in range(3):
    g.replay()
    torch.cuda.synchronize()
    try:
        print("in-graph copy ms", s0.elapsed_time(e0), flush=True)
    except Exception as ex:  # noqa: BLE001
        print("elapsed_time failed:", repr(ex), flush=True)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(); y.copy_(x); b.record(); torch.cuda.synchronize()
print("eager copy ms", a.elapsed_time(b), flush=True)
