"""Where the host time of a graph-replayed step goes (bench.py's step loop, plan lookahead 2):

    python tools/host_profile.py [--config c2] [--steps 200]

Times the enqueue of K steps with the GPU far ahead (no sync inside) and again under
cProfile; prints the enqueue us/step, the wall us/step and the top functions by own time.
"""
from __future__ import annotations

import argparse
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    import bench
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    cfg = bench.CONFIGS[a.config]
    V, F, K, B = cfg["V"], cfg["F"], cfg["K"], cfg["B"]
    dev = torch.device("cuda:0")
    torch.manual_seed(1)
    with torch.device(dev):
        m = P.FM(V, K) if cfg["kind"] == "FM" else P.DeepFM(V, F, K)
    host = list(CriteoSynth(V, F, seed=1).batches(8, B))
    xs = [torch.from_numpy(x).to(dev) for x, _ in host]
    ys = [torch.from_numpy(y).to(dev) for _, y in host]
    tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3)
    tr.flush_every = 0
    seq = [0]

    def step():
        i = seq[0]
        seq[0] += 1
        n = len(xs)
        tr.step(xs[i % n], ys[i % n], next_x=[xs[(i + 1) % n], xs[(i + 2) % n]], return_loss=False)

    for _ in range(3 * len(xs)):
        step()
    torch.cuda.synchronize()
    for rep in range(2):
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{a.config} enqueue {(t1 - t0) / a.steps * 1e6:.1f} us/step, "
              f"wall {(t2 - t0) / a.steps * 1e6:.1f} us/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
