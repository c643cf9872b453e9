"""Is the fused step host-bound? Times the Python enqueue of K steps (no sync) against the
wall time of the same K steps (sync at the end), for C2 and C3."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from rl_ctr_prediction_amd import DeepFM, FM, FusedCTRTrainer
from rl_ctr_prediction_amd.synthetic import CriteoSynth

for kind, V, F, K, B in (("FM", 1_000_000, 26, 16, 4096), ("DeepFM", 10_000_000, 26, 64, 8192)):
    dev = torch.device("cuda:0")
    torch.manual_seed(1)
    with torch.device(dev):
        m = FM(V, K) if kind == "FM" else DeepFM(V, F, K)
    xs, ys = zip(*[(torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev))
                   for x, y in CriteoSynth(V, F, seed=1).batches(4, B)])
    for mode in ("deferred", "dense"):
        tr = FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, optimizer_mode=mode)
        for i in range(5):
            tr.step(xs[i % 4], ys[i % 4])
        torch.cuda.synchronize()
        n = 30
        t0 = time.perf_counter()
        for i in range(n):
            tr.step(xs[i % 4], ys[i % 4])
        t1 = time.perf_counter()
        tr.flush()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{kind} {mode}: enqueue {((t1 - t0) / n) * 1e3:.3f} ms/step, wall "
              f"{((t2 - t0) / n) * 1e3:.3f} ms/step", flush=True)
        del tr
    del m
    torch.cuda.empty_cache()
