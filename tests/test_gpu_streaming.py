"""Streaming training: a fresh batch every step (the reference's loop,
all_main/pretrain_main.py:71-78) replays a bounded set of captured HIP graphs — every batch
is copied into a fixed input slot of its shape — and the result is bitwise the eager
launches'. Also: the bounded-staleness flush of deferred Adam, and the GC-during-capture
regression (a collection inside one trainer's capture destroying another's graphs)."""
from __future__ import annotations

import gc

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(P, kind, V, F, K, seed=8):
    torch.manual_seed(seed)
    with torch.device("cuda:0"):
        m = {"FM": lambda: P.FM(V, K), "DeepFM": lambda: P.DeepFM(V, F, K),
             "IPNN": lambda: P.InnerPNN(V, F, K)}[kind]()
    with torch.no_grad():
        m.feature_embedding.weight.mul_(0.05)
    return m


@pytest.mark.parametrize("kind,V,K,B,max_captures", [("DeepFM", 200_000, 32, 512, 8),
                                                     ("FM", 100_000, 16, 1024, 4),
                                                     ("IPNN", 100_000, 16, 256, 8)])
def test_driver_epoch_replays_bounded_graphs(cuda, kind, V, K, B, max_captures):
    """pretrain_main.train over a 20-batch epoch of distinct batches (the driver passes the
    next two batches as next_x): the step graphs are captured in the first steps only — at
    most four ((slot, planned ahead) pairs of the 3-slot ring; for the MLP kinds, whose
    weight-gradient tail is pipelined, a few more: the pending tail's slot) — and a
    second epoch captures nothing new; losses, tables and moments are bitwise the eager
    run's."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd import creat_data
    from rl_ctr_prediction_amd.pretrain_main import DeviceBatches, train
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    F = 26
    host = list(CriteoSynth(V, F, seed=5).batches(20, B))
    X = np.concatenate([x for x, _ in host])
    Y = np.concatenate([y for _, y in host])
    loader = DeviceBatches(creat_data.libsvm_dataset(X, Y), B, cuda)
    out = []
    for graphs in (False, True):
        m = _model(P, kind, V, F, K)
        tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=7)
        tr.use_graphs = graphs
        losses = []
        for epoch in range(2):
            tr.reset_optimizer()
            losses.append(train(m, tr, loader, torch.nn.BCELoss(), cuda))
            if graphs:
                if epoch == 0:
                    first = tr.captures
                    assert 1 <= first <= max_captures, first
                else:
                    assert tr.captures == first  # nothing new captured in epoch 2
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        out.append((losses, sd, tr.optimizer_state_dict()["state"]))
    (le, sde, ste), (lg, sdg, stg) = out
    assert le == lg
    for k in sde:
        assert torch.equal(sde[k], sdg[k]), k
    for i in ste:
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(ste[i][k], stg[i][k]), (i, k)


def test_fresh_batches_host_tensors_and_flush_every(cuda):
    """Host (CPU) batches are staged by the same copy; the bounded-staleness flush
    (flush_every = 3) changes no bit of the result against flush_every = 0, and leaves
    every row at most flush_every steps behind after each step."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K, B = 100_000, 26, 16, 512
    host = list(CriteoSynth(V, F, seed=9).batches(10, B))
    out = []
    for every in (0, 3):
        m = _model(P, "DeepFM", V, F, K)
        tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=7)
        tr.flush_every = every
        losses = []
        for i, (x, y) in enumerate(host):
            xb = torch.from_numpy(x) if i % 2 else torch.from_numpy(x).to(cuda)
            losses.append(tr.step(xb, torch.from_numpy(y)).item())
            if every:
                assert tr.step_count - int(tr.last.min()) <= every + 1
        out.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
        assert tr.captures == (3 if tr._pipe else 1)  # the periodic flush leaves the tail
    assert out[0][0] == out[1][0]
    for k in out[0][1]:
        assert torch.equal(out[0][1][k], out[1][1][k]), k


def test_capture_after_dropping_trainer_in_cycle(cuda):
    """Regression (commit 93faef1): trainer A, with captured graphs, dropped inside a
    reference cycle; trainer B then captures. A GC collection during B's capture would
    destroy A's graphs — HIP calls illegal while a stream captures — and abort the process;
    graph_capture collects first and pauses the collector. Runs once."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K, B = 50_000, 26, 16, 256
    (x, y), (x2, y2) = [(torch.from_numpy(a).to(cuda), torch.from_numpy(b).to(cuda))
                        for a, b in CriteoSynth(V, F, seed=2).batches(2, B)]
    m = _model(P, "DeepFM", V, F, K)
    a = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=7)
    a.step(x, y)
    a.step(x2, y2)  # A holds captured graphs
    assert a.captures >= 1
    cycle = [a, m]
    cycle.append(cycle)  # only the cyclic collector can free A now
    del a, m, cycle
    gc.disable()
    try:  # no automatic collection before B's capture starts
        m2 = _model(P, "FM", V, F, K, seed=9)
        b = P.FusedCTRTrainer(m2, lr=1e-3, weight_decay=1e-5, seed=7)
        b.step(x, y)
        loss = b.step(x2, y2).item()
    finally:
        gc.enable()
    torch.cuda.synchronize()
    assert b.captures == 1 and np.isfinite(loss)


