"""Is C2's bimodality per process or per region? Runs the bench's C2 loop (fresh batches,
plan lookahead 2, graph replay) and times R regions of K steps + the flush in ONE process:

    python tools/c2_repeat.py [--reps 6] [--steps 20] [--config c2]

Prints one line per region (M examples/s) and the trainer's stream handles.
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lookahead", type=int, default=2)
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
    n = 5 + a.reps * a.steps + 3
    host = CriteoSynth(V, F, seed=1).stream(n, B, rank=0, threads=8)
    xs = [torch.from_numpy(x).to(dev) for x, _ in host]
    ys = [torch.from_numpy(y).to(dev) for _, y in host]
    tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=1234)
    seq = [0]

    def step():
        i = seq[0]
        seq[0] += 1
        nxt = [xs[(i + j) % n] for j in range(1, a.lookahead + 1)] or None
        tr.step(xs[i % n], ys[i % n], next_x=nxt, return_loss=False)

    for _ in range(5):
        step()
    tr.flush()
    torch.cuda.synchronize()
    print("streams:", {k: getattr(tr, k).cuda_stream for k in
                       ("_side", "_plan_stream", "_capture_stream") if getattr(tr, k, None)},
          [s.cuda_stream for s in tr._extra_plan_streams], flush=True)
    for r in range(a.reps):
        t0 = time.perf_counter()
        th = 0.0
        for _ in range(a.steps):
            h = time.perf_counter()
            step()
            th += time.perf_counter() - h
        tr.flush()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"rep {r}: {B * a.steps / dt / 1e6:.2f} M ex/s, {dt / a.steps * 1e6:.1f} us/step, "
              f"host {th / a.steps * 1e6:.1f} us/step", flush=True)


if __name__ == "__main__":
    main()
