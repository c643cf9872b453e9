"""Do a C2 step graph and a sparse-plan graph overlap on the GPU? (plan lookahead A/B)

    python tools/concurrency_probe.py [--config c2] [--n 200]

Captures the trainer's graphs with step(next_x=) (a have-plan step graph and the
lookahead plan graph), then times N replays of: the step graph alone (main stream), the
plan graph alone (plan stream), and both issued together without dependencies. Prints
us per iteration for each; both ~ max(step, plan) means the two queues run concurrently.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--n", type=int, default=200)
    a = ap.parse_args()
    import bench
    from rl_ctr_prediction_amd import FM, DeepFM, FusedCTRTrainer
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    cfg = bench.CONFIGS[a.config]
    V, F, K, B = cfg["V"], cfg["F"], cfg["K"], cfg["B"]
    dev = torch.device("cuda:0")
    torch.manual_seed(1)
    with torch.device(dev):
        m = FM(V, K) if cfg["kind"] == "FM" else DeepFM(V, F, K)
    tr = FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=1)
    data = list(CriteoSynth(V, F, seed=1).batches(2, B))
    xs = [torch.from_numpy(x).to(dev) for x, _ in data]
    ys = [torch.from_numpy(y).to(dev) for _, y in data]
    for i in range(8):
        tr.step(xs[i % 2], ys[i % 2], next_x=xs[(i + 1) % 2])
    torch.cuda.synchronize()
    # a have-plan step graph (key[-1]: planned ahead) and a slot's lookahead plan graph
    g_step = next(g for key, (g, _) in tr._graphs.items() if key[-1])
    g_plan = next(s.plan_graph for ring in tr._rings.values() for s in ring
                  if s.plan_graph is not None)
    main_s = torch.cuda.current_stream()
    ps = tr._plan_stream
    out = {}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / a.n * 1e6

    out["step_us"] = timed(lambda: g_step.replay())

    def plan_only():
        with torch.cuda.stream(ps):
            g_plan.replay()
    out["plan_us"] = timed(plan_only)

    def both():
        g_step.replay()
        with torch.cuda.stream(ps):
            g_plan.replay()
    out["both_us"] = timed(both)

    def both_joined():  # lookahead 1: the next step waits for the plan just launched
        ev = torch.cuda.Event()
        ev.record(main_s)
        ps.wait_event(ev)
        g_step.replay()
        with torch.cuda.stream(ps):
            g_plan.replay()
        e2 = torch.cuda.Event()
        e2.record(ps)
        main_s.wait_event(e2)
    out["both_joined_us"] = timed(both_joined)

    ring = []

    def depth2(start_wait=True, end_wait=True):
        def fn():
            if end_wait and len(ring) >= 2:
                main_s.wait_event(ring.pop(0))
            if start_wait:
                ev = torch.cuda.Event()
                ev.record(main_s)
                ps.wait_event(ev)
            g_step.replay()
            with torch.cuda.stream(ps):
                g_plan.replay()
            e2 = torch.cuda.Event()
            e2.record(ps)
            ring.append(e2)
        return fn
    for sw, ew in ((True, True), (True, False), (False, True)):
        ring.clear()
        out[f"depth2_startwait{int(sw)}_endwait{int(ew)}_us"] = timed(depth2(sw, ew))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
