"""Is the C2 step (FM, plan lookahead two batches ahead, HIP-graph replay) host-bound?
Times the Python enqueue of K steps (no sync) against their wall time (sync at the end),
with the bench's batch sequence (bench.py step())."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from rl_ctr_prediction_amd import FM, FusedCTRTrainer
from rl_ctr_prediction_amd.synthetic import CriteoSynth

V, F, K, B = 1_000_000, 26, 16, 4096
dev = torch.device("cuda:0")
torch.manual_seed(1)
with torch.device(dev):
    m = FM(V, K)
batches = list(CriteoSynth(V, F, seed=1).batches(5, B))
xs = [torch.from_numpy(x).to(dev) for x, _ in batches]
ys = [torch.from_numpy(y).to(dev) for _, y in batches]
tr = FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=1234)
seq = [0]


def step():
    i = seq[0]
    seq[0] += 1
    return tr.step(xs[i % 5], ys[i % 5], next_x=[xs[(i + 1) % 5], xs[(i + 2) % 5]])


for _ in range(10):
    step()
torch.cuda.synchronize()
for rep in range(3):
    n = 40
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"C2 enqueue {(t1 - t0) / n * 1e6:.1f} us/step, wall {(t2 - t0) / n * 1e6:.1f} us/step",
          flush=True)
