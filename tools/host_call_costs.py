"""Host cost (us per call) of the torch / HIP calls one C2 step() makes, then a cProfile of
the C2 step loop (tools/host_overhead_c2.py's sequence)."""
import cProfile, pstats, sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

dev = torch.device("cuda:0")
s1 = torch.cuda.Stream(device=dev)
x = torch.zeros(4096, 26, dtype=torch.int64, device=dev)
ev = torch.cuda.Event()
ev.record()
g = torch.cuda.CUDAGraph()
y = torch.zeros(16, device=dev)
torch.cuda.synchronize()
with torch.cuda.graph(g):
    y.add_(1)
torch.cuda.synchronize()


def t(name, fn, n=2000):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    print(f"{name:40s} {dt:7.2f} us", flush=True)


t("torch.cuda.Event()", lambda: torch.cuda.Event())
t("ev.record()", lambda: ev.record())
t("stream.wait_event(ev)", lambda: s1.wait_event(ev))
t("x.record_stream(s1)", lambda: x.record_stream(s1))


def ctx():
    with torch.cuda.stream(s1):
        pass


t("with torch.cuda.stream(s1)", ctx)
t("torch.cuda.current_stream()", lambda: torch.cuda.current_stream())
t("g.replay() (1-node graph)", lambda: g.replay())
t("x.data_ptr()", lambda: x.data_ptr())
t("xkey", lambda: (x.data_ptr(), tuple(x.shape), x.dtype, tuple(x.stride())))
t("torch.cuda.is_current_stream_capturing()", lambda: torch.cuda.is_current_stream_capturing())

sys.argv = ["x"]
import runpy
prof = cProfile.Profile()
mod = runpy.run_path(str(Path(__file__).with_name("host_overhead_c2.py")), run_name="probe")
step = mod["step"]
prof.enable()
for _ in range(200):
    step()
prof.disable()
torch.cuda.synchronize()
pstats.Stats(prof).sort_stats("tottime").print_stats(25)
