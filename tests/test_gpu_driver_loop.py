"""The driver's epoch loop and the scratch / stream isolation of the trainers.

* The epoch loss summed on the device (fp64, inside each step's last launch) is bitwise the
  reference's per-step host sum ``total_loss += train_loss.item()``
  (all_main/pretrain_main.py:79) — for FM (the fused FM tail), DeepFM, IPNN (step_end) and
  FFM, graphs and eager.
* step() returns a fresh tensor (the reference's loss is a new tensor per step), so a list
  of returned losses is not aliased by later steps.
* The round-3 GPU memory fault (DESIGN.md §4 "Streams and scratch"): a trainer's plan
  stream handed the HIP handle of the stream its step graphs were captured on, two
  concurrent launches sharing one scratch buffer. Forced here: torch's stream pool is
  advanced to every position of its round-robin before a trainer is built, and at every
  position the trainer's streams have distinct handles and its lookahead steps stay bitwise
  the in-step plans'. Scratch is owned per trainer (hip_ops.Workspace): two trainers
  never share a buffer, whatever handles their streams got.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(P, kind, V, F, K, seed=8):
    torch.manual_seed(seed)
    with torch.device("cuda:0"):
        m = {"FM": lambda: P.FM(V, K), "DeepFM": lambda: P.DeepFM(V, F, K),
             "IPNN": lambda: P.InnerPNN(V, F, K), "FFM": lambda: P.FFM(V, F, K)}[kind]()
    if kind != "FFM":
        with torch.no_grad():
            m.feature_embedding.weight.mul_(0.05)
    return m


@pytest.mark.parametrize("kind,graphs", [("FM", True), ("DeepFM", True), ("IPNN", True),
                                         ("DeepFM", False), ("FFM", True)])
def test_driver_epoch_loss_bitwise(cuda, kind, graphs):
    """pretrain_main.train's epoch loss (device fp64 sum, one read) == the per-step
    `.item()` sum of the same steps, bit for bit; every returned loss a fresh tensor."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd import creat_data
    from rl_ctr_prediction_amd.ffm_trainer import FusedFFMTrainer
    from rl_ctr_prediction_amd.pretrain_main import DeviceBatches, train
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K, B = (20_000, 10, 8, 256) if kind == "FFM" else (100_000, 26, 16, 512)
    host = list(CriteoSynth(V, F, seed=3).batches(12, B))
    X = np.concatenate([x for x, _ in host])
    Y = np.concatenate([y for _, y in host])
    loader = DeviceBatches(creat_data.libsvm_dataset(X, Y), B, cuda)

    def trainer(m):
        if kind == "FFM":
            t = FusedFFMTrainer(m, lr=1e-3, weight_decay=1e-5)
        else:
            t = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=7)
        t.use_graphs = graphs
        return t

    # the driver's loop: two epochs (reset_optimizer between, as the driver)
    m1 = _model(P, kind, V, F, K)
    t1 = trainer(m1)
    got = []
    for _ in range(2):
        t1.reset_optimizer()
        got.append(train(m1, t1, loader, torch.nn.BCELoss(), cuda))
    # the reference's loop on a twin: per-step .item(), the returned losses kept in a list
    m2 = _model(P, kind, V, F, K)
    t2 = trainer(m2)
    want = []
    batches = list(loader)
    for _ in range(2):
        t2.reset_optimizer()
        kept, vals, total = [], [], 0.0
        for i, (x, y) in enumerate(batches):
            if kind == "FFM":
                loss = t2.step(x, y)
            else:
                loss = t2.step(x, y, next_x=[b[0] for b in batches[i + 1:i + 3]])
            kept.append(loss)
            vals.append(loss.item())
            total += vals[-1]
        want.append(total / len(batches))
        # fresh tensors: the kept losses still hold their own step's values
        assert [k.item() for k in kept] == vals
    assert got == want
    sd1, sd2 = m1.state_dict(), m2.state_dict()
    for k in sd1:
        assert torch.equal(sd1[k], sd2[k]), k


def test_returned_losses_not_aliased(cuda):
    """Losses appended over several same-shape graph-replayed steps keep their values."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K, B = 50_000, 26, 16, 256
    data = [tuple(torch.tensor(a, device=cuda) for a in xy)
            for xy in CriteoSynth(V, F, seed=4).batches(6, B)]
    tr = P.FusedCTRTrainer(_model(P, "FM", V, F, K), lr=1e-3, weight_decay=1e-5)
    losses = [tr.step(x, y) for x, y in data]
    vals = [float(l.item()) for l in losses]
    assert len(set(vals)) == len(vals)  # distinct batches: distinct losses, none overwritten
    tr2 = P.FusedCTRTrainer(_model(P, "FM", V, F, K), lr=1e-3, weight_decay=1e-5)
    assert vals == [float(tr2.step(x, y).item()) for x, y in data]


def _stream_handles(tr):
    return [s.cuda_stream for s in tr._own_streams]


@pytest.mark.parametrize("kind", ["DeepFM", "FM"])
def test_stream_pool_collision_forced(cuda, kind):
    """Advance torch's stream pool to each of its round-robin positions, then build a
    trainer: its streams always have handles of their own (none equal to another of its
    streams, the current stream, or torch's shared default capture stream), and at a few
    positions — including the one where a naive allocation would hand the plan stream the
    capture stream's handle — lookahead training is bitwise the in-step plans'."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K, B = 60_000, 26, 16, 256
    data = [tuple(torch.tensor(a, device=cuda) for a in xy)
            for xy in CriteoSynth(V, F, seed=6).batches(4, B)]
    order = [0, 1, 2, 3, 0, 1, 2, 3, 1, 0]

    def run(tr, ahead):
        out = []
        for j, i in enumerate(order):
            nxt = [data[order[k]][0] for k in range(j + 1, min(j + 1 + ahead, len(order)))]
            out.append(float(tr.step(*data[i], next_x=nxt or None).item()))
        return out, {k: v.clone() for k, v in tr.model.state_dict().items()}

    ref_tr = P.FusedCTRTrainer(_model(P, kind, V, F, K), lr=1e-3, weight_decay=1e-5, seed=7)
    ref_losses, ref_sd = run(ref_tr, 0)
    del ref_tr
    # torch's shared capture stream (what the step graphs were captured on in round 3)
    shared = getattr(torch.cuda.graph, "default_capture_stream", None)
    pool = 32  # torch's low-priority stream pool per device
    for shift in range(pool):
        for _ in range(shift):
            torch.cuda.Stream(device=cuda)
        # the handle a naive first stream of the next trainer would get
        probe = torch.cuda.Stream(device=cuda).cuda_stream
        tr = P.FusedCTRTrainer(_model(P, kind, V, F, K), lr=1e-3, weight_decay=1e-5, seed=7)
        h = _stream_handles(tr)
        assert len(set(h)) == len(h), (shift, h)
        assert torch.cuda.current_stream().cuda_stream not in h
        hit = shared is not None and shared.cuda_stream == probe
        if shift in (0, 1, 7, 31) or hit:
            losses, sd = run(tr, 2)
            h2 = _stream_handles(tr)  # plan streams created on first use: still distinct
            assert len(set(h2)) == len(h2), (shift, h2)
            assert losses == ref_losses, shift
            for k in sd:
                assert torch.equal(sd[k], ref_sd[k]), (shift, k)
        del tr


def test_scratch_owned_per_trainer(cuda):
    """Two trainers stepping in turn on one stream use disjoint scratch buffers (their own
    Workspace each), and the process-wide default owner is untouched by their steps."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd import hip_ops
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K, B = 60_000, 26, 16, 256
    x, y = (torch.tensor(a, device=cuda) for a in next(iter(CriteoSynth(V, F, seed=2).batches(1, B))))
    default = hip_ops.Workspace.current()
    t1 = P.FusedCTRTrainer(_model(P, "DeepFM", V, F, K), lr=1e-3, weight_decay=1e-5)
    t2 = P.FusedCTRTrainer(_model(P, "DeepFM", V, F, K), lr=1e-3, weight_decay=1e-5)
    before = {b.data_ptr() for b in default.buffers()}
    for _ in range(3):
        t1.step(x, y)
        t2.step(x, y)
    torch.cuda.synchronize()
    b1 = {b.data_ptr() for b in t1._scratch.buffers()}
    b2 = {b.data_ptr() for b in t2._scratch.buffers()}
    assert b1 and b2 and not (b1 & b2)
    assert {b.data_ptr() for b in default.buffers()} == before
    assert hip_ops.Workspace.current() is default  # every scope exited
