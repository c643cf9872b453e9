"""Deferred-exact dense Adam (temporal blocking) == the dense streaming pass, bitwise.

Both paths call the same per-element update with the same per-step scalars; the
deferred one replays an untouched row's g = wd*p steps in registers when the row is next
read or at flush(). Any difference — a skipped or re-ordered step, a stale read — shows
up as a bit difference in E, w, m or v.
"""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(kind, mode, V, F, K, B, batches, reset_after=None, dropout=True):
    import rl_ctr_prediction_amd as P
    torch.manual_seed(8)
    with torch.device("cuda:0"):
        m = P.FM(V, K) if kind == "FM" else P.DeepFM(V, F, K)
    if not dropout:
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
    with torch.no_grad():
        m.feature_embedding.weight.mul_(0.05)
        m.linear.weight.mul_(0.05)
    tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=7, optimizer_mode=mode)
    losses = []
    for i, (x, y) in enumerate(batches):
        if reset_after is not None and i == reset_after:
            tr.reset_optimizer()
        losses.append(tr.step(torch.tensor(x, device="cuda:0"), torch.tensor(y, device="cuda:0")).item())
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}  # state_dict flushes
    st = tr.optimizer_state_dict()["state"]
    return losses, sd, st, tr


@pytest.mark.parametrize("kind,V,K,B", [("DeepFM", 300_000, 32, 2048), ("FM", 50_000, 16, 1024),
                                        ("FM", 20_000, 10, 512)])
def test_deferred_equals_dense_bitwise(cuda, kind, V, K, B):
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    F = 26
    batches = list(CriteoSynth(V, F, seed=3).batches(9, B))
    ld, sd_d, st_d, _ = _run(kind, "dense", V, F, K, B, batches, reset_after=5)
    lf, sd_f, st_f, tr = _run(kind, "deferred", V, F, K, B, batches, reset_after=5)
    assert ld == lf
    for k in sd_d:
        assert torch.equal(sd_d[k], sd_f[k]), k
    for i in st_d:
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(st_d[i][k], st_f[i][k]), (i, k)
    assert int(tr.last.min()) == tr.step_count  # every row flushed to the last step


def test_deferred_rows_are_current_before_forward(cuda):
    """A row untouched for many steps is caught up before the next batch reads it: the
    loss of that batch equals the dense run's (it would differ with a stale row)."""
    import numpy as np
    V, F, K, B = 10_000, 4, 16, 64
    rng = np.random.default_rng(0)
    batches = []
    for i in range(12):
        x = rng.integers(0, 5000, size=(B, F))   # rows >= 5000 untouched ...
        if i == 11:
            x[:, 0] = 9999                          # ... until the last batch
        batches.append((x, (rng.random(B) < 0.3).astype(np.float32)))
    ld, sd_d, _, _ = _run("FM", "dense", V, F, K, B, batches, dropout=False)
    lf, sd_f, _, _ = _run("FM", "deferred", V, F, K, B, batches, dropout=False)
    assert ld == lf
    assert torch.equal(sd_d["feature_embedding.weight"], sd_f["feature_embedding.weight"])


@pytest.mark.parametrize("kind,mode", [("DeepFM", "deferred"), ("FM", "deferred"), ("FM", "dense"),
                                       ("DeepFM", "dense")])
def test_graph_replay_equals_eager_bitwise(cuda, kind, mode):
    """The HIP-graph replay of the step (every per-step scalar read from the device step
    counter, dropout on) produces exactly the eager launches' tables, moments and losses."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K, B = 50_000, 26, 16, 1024
    data = [(torch.tensor(x, device="cuda:0"), torch.tensor(y, device="cuda:0"))
            for x, y in CriteoSynth(V, F, seed=5).batches(3, B)]
    out = []
    for graphs in (False, True):
        torch.manual_seed(8)
        with torch.device("cuda:0"):
            m = P.FM(V, K) if kind == "FM" else P.DeepFM(V, F, K)
        m.train()
        tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=7, optimizer_mode=mode)
        tr.use_graphs = graphs
        losses = [tr.step(*data[i % 3]).item() for i in range(8)]  # 1 eager+capture, 7 replays
        if graphs:  # every batch goes through the shape's one input slot: one graph (the
            # pipelined MLP kinds: the first step's, then the slot's and the spare X plane
            # buffers alternating with the pending tail)
            n = 3 if tr._pipe else 1
            assert tr.captures == n and len(tr._graphs) == n
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        out.append((losses, sd, tr.optimizer_state_dict()["state"]))
    (le, sde, ste), (lg, sdg, stg) = out
    assert le == lg
    for k in sde:
        assert torch.equal(sde[k], sdg[k]), k
    for i in ste:
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(ste[i][k], stg[i][k]), (i, k)


@pytest.mark.parametrize("kind,K", [("FM", 16), ("FM", 32), ("DeepFM", 32), ("DeepFM", 64),
                                    ("IPNN", 32), ("IPNN", 64)])
def test_fused_scatter_apply_equals_unfused(cuda, kind, K):
    """The segmented sums with the Adam apply fused in (ctr_fm_embedding_grad_adam /
    ctr_segment_sum_rows_adam) == the separate sums + ctr_adam_deferred_rows, bitwise — the
    tables, the moments and (keep_grads) the per-row sums — on Zipf batches whose hot rows
    span many chunks. K 16 / 32 / 64: 16 / 8 / 4 rows per wave in the fused pass, so both
    of its spanning-row paths (a row's own lane group, the whole wave for hot rows) run."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, B = 200_000, 26, 2048
    batches = list(CriteoSynth(V, F, seed=5).batches(6, B))
    out = []
    for fuse in (False, True):
        torch.manual_seed(8)
        with torch.device("cuda:0"):
            m = {"FM": lambda: P.FM(V, K), "DeepFM": lambda: P.DeepFM(V, F, K),
                 "IPNN": lambda: P.InnerPNN(V, F, K)}[kind]()
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
        with torch.no_grad():
            m.feature_embedding.weight.mul_(0.05)
        tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=7)
        tr.fuse_apply, tr.keep_grads = fuse, True
        for x, y in batches:
            tr.step(torch.tensor(x, device="cuda:0"), torch.tensor(y, device="cuda:0"))
        U = tr._bufs.plan.num_unique_host()
        grads = (tr._bufs.grad_rows[:U].clone(), tr._bufs.grad_lin[:U].clone())
        out.append(({k: v.detach().clone() for k, v in m.state_dict().items()},
                    tr.optimizer_state_dict()["state"], grads))
    (sd0, st0, g0), (sd1, st1, g1) = out
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k
    for i in st0:
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(st0[i][k], st1[i][k]), (i, k)
    assert torch.equal(g0[0], g1[0])
    if kind != "IPNN":
        assert torch.equal(g0[1], g1[1])


def test_c3_full_size_deferred_equals_dense_20_steps(cuda):
    """C3 at full size (DeepFM, V = 10M, K = 64, B = 8192, dropout 0.2) over the bench's
    region length — 20 steps on 4 cycled batches after a 3-step warm-up and flush, as
    bench.py times it: deferred-exact Adam == the dense streaming pass, bitwise, on the
    losses, the dense parameters, and p / m / v of the touched rows and 200k sampled rows."""
    import gc

    import numpy as np
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K, B = 10_000_000, 26, 64, 8192
    host = list(CriteoSynth(V, F, seed=11).batches(4, B))
    batches = [(torch.tensor(x, device=cuda), torch.tensor(y, device=cuda)) for x, y in host]
    rng = np.random.default_rng(2)
    touched = np.unique(np.concatenate([x.reshape(-1) for x, _ in host]))
    sample = torch.tensor(np.unique(np.concatenate([touched, rng.integers(0, V, 200_000),
                                                    [0, V - 1]])), device=cuda)
    out = {}
    for mode in ("deferred", "dense"):
        torch.manual_seed(4)
        with torch.device("cuda:0"):
            m = P.DeepFM(V, F, K)
        with torch.no_grad():
            m.feature_embedding.weight.mul_(0.05)
            m.linear.weight.mul_(0.05)
        tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=1234, optimizer_mode=mode)
        for i in range(3):
            tr.step(*batches[i % 4])
        tr.flush()
        losses = [tr.step(*batches[i % 4]).item() for i in range(20)]
        tr.flush()
        out[mode] = dict(losses=losses,
                         E=m.feature_embedding.weight.detach()[sample].cpu(),
                         w=m.linear.weight.detach()[sample].cpu(),
                         mE=tr.m_E[sample].cpu(), vE=tr.v_E[sample].cpu(),
                         mw=tr.m_w[sample].cpu(), vw=tr.v_w[sample].cpu(),
                         dense={k: v.detach().cpu().clone() for k, v in tr.views.items()})
        if mode == "deferred":
            assert int(tr.last.min()) == tr.step_count == 23
        del tr, m
        gc.collect()
        torch.cuda.empty_cache()
    a, b = out["deferred"], out["dense"]
    assert a["losses"] == b["losses"]
    for k in ("E", "w", "mE", "vE", "mw", "vw"):
        assert torch.equal(a[k], b[k]), k
    for k in a["dense"]:
        assert torch.equal(a["dense"][k], b["dense"][k]), k


@pytest.mark.parametrize("kind,V,K,B", [("FM", 50_000, 16, 1024), ("DeepFM", 200_000, 32, 1024),
                                        ("IPNN", 100_000, 16, 512)])
def test_plan_lookahead_bitwise(cuda, kind, V, K, B):
    """step(x, y, next_x=...) stages the next batches and builds their plans during this
    step (one or two ahead, the second one a guess the order sometimes breaks): bitwise the same
    losses, tables and moments as building every plan in its own step — over graph captures
    and replays, a lookahead the next step does not use (order changed), next_x == x, a step
    without next_x in between, eager (no-graph) steps, and labels staged with next_y (the
    batch's own: its label copy skipped; a decoy: its own labels still copied)."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    F = 26
    data = list(CriteoSynth(V, F, seed=5).batches(3, B))
    xs = [torch.tensor(x, device=cuda) for x, _ in data]
    ys = [torch.tensor(y, device=cuda) for _, y in data]
    # (batch, next batch or None) per step: cycles (captured, then replayed), a skipped
    # lookahead (next 2, then batch 1), next == x, no next, then cycles again
    order = [(0, 1), (1, 2), (2, 0), (0, 1), (1, 2), (2, 0), (0, 2), (1, 1), (1, None),
             (2, 0), (0, 1), (1, 2), (2, 0), (0, 1)]
    decoy = [1.0 - y for y in ys]  # staged labels the steps then do not train on
    out = []
    # (batches ahead, HIP graphs, plan lookahead, labels staged too: None / the batch's own
    # (its step skips the label copy) / a decoy (its step must copy its own y))
    # (+ pig: the next batch's plan built inside the step's graph, plan_in_graph)
    for ahead, graphs, pla, ymode, pig_on in (
            (0, True, False, None, False), (1, True, True, None, False),
            (2, True, True, None, False), (2, False, True, None, False),
            (2, True, False, None, False), (1, False, True, None, False),
            (2, True, True, "own", False), (1, False, True, "own", False),
            (2, True, True, "decoy", False), (2, True, True, None, True),
            (1, True, True, "own", True), (2, False, True, None, True)):
        torch.manual_seed(8)
        with torch.device(cuda):
            m = {"FM": lambda: P.FM(V, K), "DeepFM": lambda: P.DeepFM(V, F, K),
                 "IPNN": lambda: P.InnerPNN(V, F, K)}[kind]()
        with torch.no_grad():
            m.feature_embedding.weight.mul_(0.05)
        tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=7)
        tr.use_graphs = graphs
        tr.plan_lookahead = pla  # default: FM only; exercised for every kind here
        tr.plan_in_graph = pig_on
        losses = []
        for j, (i, n) in enumerate(order):
            nxt = xs[n] if (ahead and n is not None) else None
            nb = [n] if (ahead and n is not None) else []
            if ahead == 2 and n is not None:  # the next two batches of the order
                nb = [n] + ([order[j + 2][0]] if j + 2 < len(order) else [])
                nxt = [xs[q] for q in nb]
            nyt = None
            if ymode is not None and nb:
                nyt = [(ys if ymode == "own" else decoy)[q] for q in nb]
            losses.append(tr.step(xs[i], ys[i], next_x=nxt, next_y=nyt).item())
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        st = tr.optimizer_state_dict()["state"]
        out.append((losses, sd, st))
        if graphs:  # (slot, planned ahead) pairs of a ring of ahead + 1 slots (x the
            # pipelined kinds' X plane buffer and pending-tail variants; x the slot whose
            # plan the step builds in its graph — one of the ring or none — for the MLP kinds)
            pig = tr.plan_in_graph and ahead > 0 and pla
            assert tr.captures <= 2 * (ahead + 1) * (3 if tr._pipe else 1) * (
                (ahead + 2) if pig else 1)
    for losses, sd, st in out[1:]:
        assert losses == out[0][0]
        for k in sd:
            assert torch.equal(sd[k], out[0][1][k]), k
        for i in st:
            for k in ("exp_avg", "exp_avg_sq"):
                assert torch.equal(st[i][k], out[0][2][i][k]), (i, k)


@pytest.mark.parametrize("K,V,T,lin", [(64, 100_003, 23, True), (16, 100_003, 23, True),
                                       (8, 100_003, 23, True), (128, 100_003, 23, True),
                                       (10, 100_003, 23, True), (64, 37, 5, True),
                                       (32, 70_001, 300, False), (256, 4_099, 9, True)])
def test_flush_tile_equals_scalar_bitwise(cuda, K, V, T, lin):
    """The tiled flush (deferred_flush_tile: 64-row tiles, float4 columns, K % 4 == 0) ==
    the thread-per-row kernel (deferred_scalar, taken for tables that are not 16-B aligned),
    bitwise, on rows of mixed staleness (current, 1 step, up to the full region), a row
    count that is not a multiple of 64 (and one below 64), steps older than any LDS window
    (T = 300) and a table without linear weights."""
    from rl_ctr_prediction_amd import hip_ops as H
    g = torch.Generator(device=cuda).manual_seed(K + V)
    E0 = torch.randn(V, K, device=cuda, generator=g) * 0.05
    m0 = torch.randn(V, K, device=cuda, generator=g) * 1e-4
    v0 = torch.rand(V, K, device=cuda, generator=g) * 1e-8
    w0 = torch.randn(V, device=cuda, generator=g) * 0.05
    last0 = torch.randint(0, T + 1, (V,), device=cuda, generator=g, dtype=torch.int32)
    last0[:min(640, V // 2)] = T  # whole tiles already current

    def shifted(t):  # the same values at a 4-B (not 16-B) aligned address
        buf = torch.empty(t.numel() + 1, device=cuda)
        out = buf[1:].view(t.shape)
        out.copy_(t)
        return out

    tab = H.AdamStepTable(1e-3, (0.9, 0.999), cuda)
    out = []
    for aligned in (True, False):
        mk = (lambda t: t.clone()) if aligned else shifted
        E, m, v = mk(E0), mk(m0), mk(v0)
        w = w0.clone()
        mw, vw, last = torch.zeros_like(w), torch.zeros_like(w), last0.clone()
        if lin:
            H.adam_deferred_flush(E, m, v, w, mw, vw, last, T, tab, weight_decay=1e-5)
        else:
            H.adam_deferred_flush(E, m, v, None, None, None, last, T, tab, weight_decay=1e-5)
        out.append((E, m, v, w, mw, vw, last))
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)
    assert int(out[0][6].min()) == T


@pytest.mark.parametrize("kind", ["DeepFM", "IPNN"])
@pytest.mark.parametrize("graphs", [True, False])
def test_pipelined_wgrad_tail_bitwise(cuda, kind, graphs):
    """The MLP weight-gradient tail pipelined into the next step (dW0 + the MLP Adam at
    the start of step t+1, beside its catch-up and gather; trainer._pipe) gives bitwise the
    unpipelined trainer's losses, parameters and moments: over ragged batch shapes (the
    tail of one shape applied in a step of another), plans built ahead on some steps,
    periodic table flushes (which leave the tail pending), a state_dict read in the middle
    (which applies it) and dropout on."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K = 60_000, 26, 32
    sizes = [512, 512, 300, 512, 512, 512, 300, 300, 512]
    data = [tuple(torch.tensor(a, device=cuda) for a in xy)
            for xy in (next(iter(CriteoSynth(V, F, seed=40 + i).batches(1, b)))
                       for i, b in enumerate(sizes))]
    out = {}
    for piped in (False, True):
        torch.manual_seed(8)
        with torch.device("cuda:0"):
            m = P.DeepFM(V, F, K) if kind == "DeepFM" else P.InnerPNN(V, F, K)
        tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=7)
        tr._pipe = piped  # (opt-in: CTR_PIPELINE_WGRAD=1)
        tr.use_graphs = graphs
        tr.flush_every = 3
        losses, mid = [], None
        for i, (x, y) in enumerate(data):
            nxt = [d[0] for d in data[i + 1:i + 3]] if i % 4 != 1 else None
            losses.append(tr.step(x, y, next_x=nxt).item())
            if i == 4:
                mid = {k: v.detach().clone() for k, v in m.state_dict().items()}
            if piped and i == 5:
                assert tr._tail is not None  # pending between steps
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        assert tr._tail is None
        st = tr.optimizer_state_dict()["state"]
        out[piped] = (losses, mid, sd, st)
    a, b = out[False], out[True]
    assert a[0] == b[0]
    for d1, d2 in ((a[1], b[1]), (a[2], b[2])):
        for k in d1:
            assert torch.equal(d1[k], d2[k]), k
    for i in a[3]:
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(a[3][i][k], b[3][i][k]), (i, k)
