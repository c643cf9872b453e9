"""Row-sharded data parallelism (rl_ctr_prediction_amd/sharded.py) on the GPU.

* world size 1: every exchange is a local copy, so the sharded step must equal the
  single-GPU FusedCTRTrainer step bitwise (tables, moments, losses);
* world size 2 on one GPU (gloo, the collectives staged through the host): two ranks
  training their halves of a global batch must match one process training the whole
  batch, within the fp32 bar — the per-row gradient is summed per rank and then across
  ranks (another association order than one process's chunked sum), the dense MLP
  gradient likewise through the all-reduce. The parameters are checked element by element
  against conftest.AdamBound, built from the one-process run's per-step gradients and the
  gradient bar (assert_grad_close's, with the oracle's condition numbers), which is
  assumed for the ranks' gradients here and checked directly against the oracle in
  test_gpu_models.
"""
from __future__ import annotations

import gc
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import collect_ranks, AdamBound, fused_grads, grad_bound

pytestmark = pytest.mark.gpu


def _model(kind, V, F, K, seed=4, drop=0.0, device="cuda:0"):
    import rl_ctr_prediction_amd as P
    torch.manual_seed(seed)
    with torch.device(device):
        m = {"FM": lambda: P.FM(V, K), "DeepFM": lambda: P.DeepFM(V, F, K),
             "IPNN": lambda: P.InnerPNN(V, F, K)}[kind]()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = drop
    with torch.no_grad():
        m.feature_embedding.weight.mul_(0.05)
        if kind != "IPNN":
            m.linear.weight.mul_(0.05)
    return m


@pytest.mark.parametrize("kind,V,K,B", [("FM", 40_000, 16, 1024), ("DeepFM", 200_000, 32, 2048),
                                        ("IPNN", 200_000, 32, 2048)])
def test_sharded_world1_equals_fused_bitwise(cuda, kind, V, K, B):
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    F = 26
    batches = list(CriteoSynth(V, F, seed=11).batches(6, B))
    out = {}
    for name in ("fused", "padded", "varsplit"):
        m = _model(kind, V, F, K)
        if name == "fused":
            tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3, optimizer_mode="deferred")
        else:
            tr = P.ShardedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3, exchange=name)
        xs = [torch.tensor(x, device=cuda) for x, _ in batches]
        ys = [torch.tensor(y, device=cuda) for _, y in batches]
        # the sharded runs build their plans two batches ahead (next_x), the fused one in-step
        losses = [tr.step(xs[i], ys[i], next_x=(xs[i + 1:i + 3] if name != "fused"
                                                 else None)).item()
                  for i in range(len(xs))]
        if name == "padded":  # the fixed-capacity step replays captured graphs at N = 1;
            # the capacity only grows, and the buffers / graphs of a smaller one are dropped
            assert 1 <= tr.captures <= 6 and 1 <= len(tr._graphs) <= tr.captures
            assert len(tr._xbufs) == 1 and all(k[2] == tr._cap for k in tr._xbufs)
        tr.check_errors()
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        st = tr.optimizer_state_dict()["state"]
        out[name] = (losses, sd, st)
    lf, sdf, stf = out["fused"]
    for name in ("padded", "varsplit"):
        ls, sds, sts = out[name]
        assert lf == ls, name
        for k in sdf:
            assert torch.equal(sdf[k], sds[k]), (name, k)
        for i in stf:
            for k in ("exp_avg", "exp_avg_sq"):
                assert torch.equal(stf[i][k], sts[i][k]), (name, i, k)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, kind, V, F, K, B, steps, q, drop=0.0, exchange="padded",
               layout="cyclic"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rl_ctr_prediction_amd as P
        from rl_ctr_prediction_amd.synthetic import CriteoSynth
        torch.cuda.set_device(0)
        m = _model(kind, V, F, K, drop=drop)
        tr = P.ShardedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3, exchange=exchange,
                                 layout=layout)
        # the rank holds its row shard only: blocks ceil(V/N) rows (the last rank the
        # remainder), cyclic the rows r, r + N, r + 2N, ...
        Vs = -(-V // world)
        rows = min(Vs, V - rank * Vs) if layout == "blocks" else len(range(rank, V, world))
        E_loc = m.feature_embedding.weight
        # (+ one spare row: the fixed-capacity exchange's padding target)
        assert tuple(E_loc.shape) == (rows, K) and tr.V_tab == rows
        assert E_loc.untyped_storage().nbytes() == (rows + 1) * K * 4
        assert tr.m_E.shape[0] == tr.v_E.shape[0] == tr.last.shape[0] == rows + 1
        if kind != "IPNN":
            assert m.linear.weight.untyped_storage().nbytes() == (rows + 1) * 4
        losses = []
        data = [(torch.tensor(x[rank * B:(rank + 1) * B], device="cuda:0"),
                 torch.tensor(y[rank * B:(rank + 1) * B], device="cuda:0"))
                for x, y in CriteoSynth(V, F, seed=21).batches(steps, B * world)]
        for i, (xs, ys) in enumerate(data):
            # odd ranks build their plans ahead (next_x), even ranks in-step: a local choice
            nxt = [d[0] for d in data[i + 1:i + 3]] if rank % 2 == 1 else None
            losses.append(tr.step(xs, ys, next_x=nxt).item())
        E, w = tr.gather_tables()
        sd = tr.full_state_dict()  # every rank: the full tables are gathered into it
        assert torch.equal(sd["feature_embedding.weight"], E)
        # model.state_dict() is local (no collective): rank 0 alone may save it, and every
        # rank resumes from its own dict or from the full one (cut to its rows)
        import io
        buf = io.BytesIO()
        torch.save(m.state_dict(), buf)  # the shard, its row range in the metadata
        buf.seek(0)
        local = torch.load(buf, weights_only=True)
        assert local["feature_embedding.weight"].shape[0] == rows
        assert list(local._metadata[""]["ctr_rows"]) == tr.shard_meta()
        assert tr.shard_meta() == (["cyclic", rank, world, V] if layout == "cyclic" else
                                   [rank * Vs, rank * Vs + rows, V])
        # another rank's shard (equal shard sizes here) or a shard without its row range is
        # refused, not loaded as this rank's rows
        other = [None] * world
        dist.all_gather_object(other, buf.getvalue())
        theirs = torch.load(io.BytesIO(other[(rank + 1) % world]), weights_only=True)
        with pytest.raises(RuntimeError, match="row range"):
            m.load_state_dict(theirs)
        with pytest.raises(RuntimeError, match="row range"):
            m.load_state_dict(dict(local))  # a plain dict: no metadata
        dist.barrier()
        m.load_state_dict(local)
        m.load_state_dict(sd)
        after = m.state_dict()
        for k in local:
            assert torch.equal(after[k], local[k]), k
        Ec, wc = tr.gather_tables(device="cpu")  # shard by shard, into host memory
        assert torch.equal(Ec, E.cpu())
        # this rank's rows of the full table are its shard (the layout's row order)
        assert torch.equal(tr._cut(E), m.feature_embedding.weight.detach())
        if w is not None:
            assert torch.equal(sd["linear.weight"], w) and torch.equal(wc, w.cpu())
        with pytest.raises(RuntimeError, match="row shard"):
            m(data[0][0])
        dense = {k: v.detach().cpu().numpy() for k, v in sd.items()
                 if k not in ("feature_embedding.weight", "linear.weight")}
        # numpy, pickled by value: a torch tensor would travel as a shared-memory fd that the
        # parent can only open while this process is still alive
        q.put((rank, losses, E.cpu().numpy(), None if w is None else w.cpu().numpy(), dense))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,drop,V,F,K,B", [
    ("FM", 0.0, 30_000, 26, 16, 512), ("DeepFM", 0.0, 30_000, 26, 16, 512),
    ("DeepFM", 0.2, 30_000, 26, 16, 512), ("IPNN", 0.0, 30_000, 26, 16, 512),
    # C5's row shape (Avazu 22 fields, dim 128): both shards own hot rows
    ("FM", 0.0, 200_000, 22, 128, 1024)])
def test_sharded_world2_matches_global_batch(cuda, kind, drop, V, F, K, B):
    """drop > 0: the dropout masks are drawn from the global-batch element index, so the two
    ranks' masks are the halves of the one-process global-batch masks (not two copies of
    rank 0's), and the runs agree within the bar with dropout on. Cyclic row ownership (the
    default layout)."""
    _check_global_batch(cuda, kind, drop, V, F, K, B, world=2, min_share=0.05)


@pytest.mark.parametrize("kind", ["DeepFM", "FM"])
def test_sharded_world2_blocks_layout_matches_global_batch(cuda, kind):
    """The contiguous-blocks layout (layout="blocks": rank r owns [r*Vs, (r+1)*Vs)) against
    the same one-process global-batch run."""
    _check_global_batch(cuda, kind, 0.0, 30_000, 26, 16, 512, world=2, min_share=0.05,
                        layout="blocks")


@pytest.mark.parametrize("kind,drop,V,F,K,B", [
    ("DeepFM", 0.2, 60_000, 26, 16, 512), ("FM", 0.0, 200_000, 22, 128, 1024)])
def test_sharded_world4_matches_global_batch(cuda, kind, drop, V, F, K, B):
    """Four ranks (gloo, one GPU): every owner receives four runs per step (one per
    requester, its own included), so the owners' runs plan, the entry sums over up to four
    sources and the three all-to-alls run past the two-rank case; the ranks' tables, dense
    parameters and losses match one process on the global batch within the bar."""
    _check_global_batch(cuda, kind, drop, V, F, K, B, world=4, min_share=0.04)


def _check_global_batch(cuda, kind, drop, V, F, K, B, world, min_share, layout="cyclic"):
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    steps = 4
    # every shard owns hot rows (>= 100 hits over the run) and >= min_share of the slots: the
    # exchange carries real traffic every way
    xs = np.concatenate([x for x, _ in CriteoSynth(V, F, seed=21).batches(steps, B * world)])
    ids, cnt = np.unique(xs, return_counts=True)
    owner = ids // -(-V // world) if layout == "blocks" else ids % world
    for r in range(world):
        assert cnt[owner == r].max() >= 100, (r, cnt[owner == r].max())
        assert cnt[owner == r].sum() >= min_share * xs.size, (r, cnt[owner == r].sum() / xs.size)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main,
                         args=(r, world, port, kind, V, F, K, B, steps, q, drop, "padded", layout))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for r in collect_ranks(procs, q, world):
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # one process, the whole global batch; its per-step gradients and their bar build the
    # per-element Adam interval the ranks' parameters must fall in
    from oracle import ctr_oracle as O
    m = _model(kind, V, F, K, drop=drop)
    tr = P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3)
    tr.keep_grads = True  # fused_grads reads the per-row sums
    sd = m.state_dict()
    bd = {k: AdamBound(v.cpu().numpy(), 1e-3, 1e-5) for k, v in sd.items()}
    ref_losses = []
    for x, y in CriteoSynth(V, F, seed=21).batches(steps, B * world):
        cpu = {k: v.detach().cpu() for k, v in m.state_dict().items()}
        cond = O.grad_condition(kind, cpu, torch.tensor(x), torch.tensor(y))
        ref_losses.append(tr.step(torch.tensor(x, device=cuda),
                                  torch.tensor(y, device=cuda)).item())
        gE, gw, dense = fused_grads(tr)
        n = np.bincount(np.asarray(x).reshape(-1), minlength=V)
        grads = dict(dense, **{"feature_embedding.weight": gE})
        if gw is not None:
            grads["linear.weight"] = gw
        for k, g in grads.items():
            c = cond.get(k)
            bd[k].step(g, grad_bound(g, cond=None if c is None else c.numpy(),
                                     n_terms=None if c is None else n))
    tr.flush()
    sd = m.state_dict()
    for rank in range(world):
        losses, E, w, dense = res[rank]
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-5)
        bd["feature_embedding.weight"].check(E, sd["feature_embedding.weight"].cpu().numpy(),
                                             err_msg=f"E rank {rank}")
        if w is not None:
            bd["linear.weight"].check(w, sd["linear.weight"].cpu().numpy(),
                                      err_msg=f"w rank {rank}")
        for k, v in dense.items():
            bd[k].check(v, sd[k].cpu().numpy(), err_msg=f"{k} rank {rank}")
    # the replicated dense parameters are bitwise identical across ranks
    for r in range(1, world):
        for k in res[0][3]:
            assert np.array_equal(res[0][3][k], res[r][3][k]), (r, k)


def _host_rank_main(rank, world, port, V, F, K, B, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rl_ctr_prediction_amd as P
        torch.cuda.set_device(0)
        torch.manual_seed(7)
        m = P.DeepFM(V, F, K)  # on the host: the reference's own init (CPU generator)
        init = m.feature_embedding.weight.detach().clone()
        tr = P.ShardedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3, device="cuda:0")
        shard = m.feature_embedding.weight.detach().cpu()
        assert torch.equal(shard, init[rank::world])  # the reference init's rows (cyclic), bitwise
        assert m.mlp[0].weight.is_cuda
        g = torch.Generator().manual_seed(rank)
        x = torch.randint(0, V, (B, F), generator=g).cuda()
        y = (torch.rand(B, generator=g) < 0.3).float().cuda()
        loss = tr.step(x, y).item()
        q.put((rank, float(loss)))
    finally:
        dist.destroy_process_group()


def test_sharded_model_built_on_host(cuda):
    """A model built on the host (the reference's CPU init) is sharded straight to the
    device: each rank's shard holds exactly the init's rows [lo, hi), no full table is
    ever placed on the GPU, and a step trains."""
    world, V, F, K, B = 2, 50_000, 8, 16, 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_rank_main, args=(r, world, port, V, F, K, B, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(collect_ranks(procs, q, world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1] and np.isfinite(res[0])  # the loss is all-reduced: equal


def _ab_rank_main(rank, world, port, kind, V, F, K, B, steps, q, backend="gloo", graphs=None):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if graphs is not None:
        os.environ["CTR_SHARDED_GRAPHS"] = "1" if graphs else "0"
    dev = torch.device("cuda", rank if backend == "nccl" else 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rl_ctr_prediction_amd as P
        from rl_ctr_prediction_amd.synthetic import CriteoSynth
        data = [(torch.tensor(x[rank * B:(rank + 1) * B], device=dev),
                 torch.tensor(y[rank * B:(rank + 1) * B], device=dev))
                for x, y in CriteoSynth(V, F, seed=23).batches(steps, B * world)]
        res = {}
        for exchange in ("padded", "varsplit"):
            m = _model(kind, V, F, K, drop=0.2, device=dev)
            tr = P.ShardedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3, exchange=exchange)
            losses = []
            for i, (xs, ys) in enumerate(data):
                nxt = [d[0] for d in data[i + 1:i + 3]] if (rank + i) % 3 else None
                losses.append(tr.step(xs, ys, next_x=nxt).item())
            tr.check_errors()
            E, w = tr.gather_tables()
            res[exchange] = (losses, E.cpu().numpy(), None if w is None else w.cpu().numpy(),
                             {k: v.detach().cpu().numpy() for k, v in tr.views.items()},
                             tr.m_E[:tr.V_tab].cpu().numpy(), tr.v_E[:tr.V_tab].cpu().numpy())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,K", [("DeepFM", 16), ("FM", 32), ("IPNN", 16)])
def test_padded_exchange_equals_varsplit_world2(cuda, kind, K):
    """The fixed-capacity exchange (equal-split all-to-alls padded to the agreed capacity,
    the spare-row padding) gives bitwise the variable-split protocol's tables, moments,
    dense parameters and losses at world size 2 (gloo), dropout on, plans built ahead on
    some steps and in-step on others, differently on the two ranks."""
    world, V, F, B, steps = 2, 40_000, 26, 512, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ab_rank_main, args=(r, world, port, kind, V, F, K, B, steps, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(collect_ranks(procs, q, world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        a, b = res[rank]["padded"], res[rank]["varsplit"]
        assert a[0] == b[0], rank
        for x, y in ((a[1], b[1]), (a[2], b[2]), (a[4], b[4]), (a[5], b[5])):
            if x is not None:
                assert np.array_equal(x, y), rank
        for k in a[3]:
            assert np.array_equal(a[3][k], b[3][k]), (rank, k)


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs two GPUs (RCCL over xGMI)")
@pytest.mark.parametrize("graphs", [False, True])
def test_padded_exchange_equals_varsplit_world2_rccl(cuda, graphs):
    """The same A/B as test_padded_exchange_equals_varsplit_world2 over RCCL (backend
    nccl, one GPU per rank), eager and with the collectives captured in the step graphs
    (CTR_SHARDED_GRAPHS=1): pins the exchange under real all_to_all_single. Skipped on the
    one-GPU boxes of this pool (the RCCL path is unverified until it runs)."""
    world, V, F, K, B, steps = 2, 40_000, 26, 16, 512, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ab_rank_main,
                         args=(r, world, port, "DeepFM", V, F, K, B, steps, q, "nccl", graphs))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(collect_ranks(procs, q, world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        a, b = res[rank]["padded"], res[rank]["varsplit"]
        assert a[0] == b[0], rank
        for x, y in ((a[1], b[1]), (a[2], b[2]), (a[4], b[4]), (a[5], b[5])):
            if x is not None:
                assert np.array_equal(x, y), rank
        for k in a[3]:
            assert np.array_equal(a[3][k], b[3][k]), (rank, k)


@pytest.mark.parametrize("depth", [1, 2])
def test_capacity_read_never_waits_for_main(cuda, depth):
    """The row-sharded step's one host read (the agreed exchange capacity) never waits for
    work enqueued on the main stream after the previous step() call: with a long sleep
    kernel queued on the main stream between two calls, step() returns while the sleep still
    runs. Run in the suite's own process, after every other test here has created its
    streams: the agreement a step reads is enqueued by an earlier call (at its end), so in
    FIFO order it precedes the sleep on whichever hardware queue its stream shares
    (the stream-to-queue mapping)."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K, B = 50_000, 26, 16, 512
    data = [tuple(torch.tensor(a, device=cuda) for a in xy)
            for xy in CriteoSynth(V, F, seed=12).batches(4, B)]
    tr = P.ShardedCTRTrainer(_model("FM", V, F, K), lr=1e-3, weight_decay=1e-5, seed=3)

    def nxt(i):
        return [data[(i + j) % 4][0] for j in range(1, depth + 1)]

    for i in range(12):  # every (slot, capacity) graph captured
        tr.step(*data[i % 4], next_x=nxt(i), return_loss=False)
    torch.cuda.synchronize()
    reads, blocking = tr.cap_reads, tr.cap_blocking
    assert blocking == 1  # the first step only: nothing was agreed before it
    main = torch.cuda.current_stream()
    torch.cuda._sleep(600_000_000)  # 0.25-6 s of one wave spinning on the main stream
    after_sleep = torch.cuda.Event()
    after_sleep.record(main)
    t0 = time.perf_counter()
    tr.step(*data[0], next_x=nxt(12), return_loss=False)
    host_s = time.perf_counter() - t0
    pending = not after_sleep.query()
    torch.cuda.synchronize()
    sleep_s = time.perf_counter() - t0
    r = dict(reads=tr.cap_reads - reads, blocking=tr.cap_blocking - blocking,
             pending=pending, host_s=host_s, sleep_s=sleep_s)
    assert r["reads"] == 1 and r["blocking"] == 0, r
    assert r["pending"], f"step() waited for the main stream: {r}"


def test_capacity_agreement_mismatch(cuda):
    """A step whose batch is not the one announced for it (next_x) is agreed in the step
    (one process; with collectives the ranks sized the step by the announced batch and the
    step raises instead); steps without lookahead agree in the step, and every result is
    bitwise the fused trainer's."""
    import rl_ctr_prediction_amd as P
    from rl_ctr_prediction_amd.synthetic import CriteoSynth
    V, F, K, B = 50_000, 26, 16, 512
    data = [tuple(torch.tensor(a, device=cuda) for a in xy)
            for xy in CriteoSynth(V, F, seed=13).batches(6, B)]
    out = {}
    for name in ("fused", "sharded"):
        m = _model("FM", V, F, K)
        tr = (P.FusedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3) if name == "fused" else
              P.ShardedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3))
        # announced 1, 2; then 5 trains instead of 2 (a decoy), no lookahead, then 3, 4:
        # agreed in the step at calls 0 (first), 2 (decoy), 3 and 5 (nothing announced)
        order = [(0, [1, 2]), (1, [2]), (5, None), (3, [4]), (4, None), (2, [0])]
        losses = [tr.step(*data[i], next_x=None if n is None else [data[j][0] for j in n]
                          ).item() for i, n in order]
        tr.flush()
        out[name] = (losses, m.feature_embedding.weight.detach().clone())
        if name == "sharded":
            assert tr.cap_reads == len(order) and tr.cap_blocking == 4, (
                tr.cap_reads, tr.cap_blocking)
    assert out["fused"][0] == out["sharded"][0]
    assert torch.equal(out["fused"][1], out["sharded"][1])


def _rccl_world1_main(q, port, kind, V, F, K, B, steps, name, force, graphs):
    import sys
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        import rl_ctr_prediction_amd as P
        from rl_ctr_prediction_amd.synthetic import CriteoSynth
        data = [tuple(torch.tensor(a, device=dev) for a in xy)
                for xy in CriteoSynth(V, F, seed=31).batches(steps, B)]
        m = _model(kind, V, F, K, drop=0.2, device=dev)
        tr = P.ShardedCTRTrainer(m, lr=1e-3, weight_decay=1e-5, seed=3, force_collectives=force)
        tr.use_graphs = graphs
        losses = []
        for i in range(steps):
            losses.append(tr.step(*data[i], next_x=[d[0] for d in data[i + 1:i + 3]]).item())
            print(f"[rccl {name}] step {i} done", file=sys.stderr, flush=True)
        tr.check_errors()
        E, w = tr.gather_tables()
        res = dict(losses=losses, E=E.cpu().numpy(), w=None if w is None else w.cpu().numpy(),
                   dense={k: v.detach().cpu().numpy() for k, v in tr.views.items()},
                   m=tr.m_E[:tr.V_tab].cpu().numpy(), v=tr.v_E[:tr.V_tab].cpu().numpy(),
                   captures=tr.captures, blocking=tr.cap_blocking,
                   backend=dist.get_backend(tr.group))
        # the captured graphs (RCCL kernels inside) go before the communicators do
        torch.cuda.synchronize()
        del tr, m, E, w
        gc.collect()
        q.put(res)
    finally:
        torch.cuda.synchronize()
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,K", [("DeepFM", 16), ("FM", 32)])
def test_rccl_world1_collectives_bitwise(cuda, kind, K):
    """RCCL on the hardware: the row-sharded step with every exchange sent through the
    collectives of a one-rank nccl (RCCL) process group — equal-split all_to_all_single for
    ids / rows / gradients, all_reduce for the dense gradient, the loss and the capacity
    agreements — eager and captured into the step's HIP graphs, is bitwise the local-copy
    step over 5 steps with two batches of lookahead (dropout on). Each variant in a process
    of its own (one communicator set per process), bounded well inside the suite's limits."""
    V, F, B, steps = 40_000, 26, 512, 5
    ctx = mp.get_context("spawn")
    res = {}
    for name, force, graphs in (("local", False, True), ("rccl_eager", True, False),
                                ("rccl_graphs", True, True)):
        q = ctx.Queue()
        p = ctx.Process(target=_rccl_world1_main,
                        args=(q, _free_port(), kind, V, F, K, B, steps, name, force, graphs))
        p.start()
        try:
            res[name] = q.get(timeout=90)
            p.join(timeout=30)
        finally:
            if p.is_alive():  # never leave a rank behind on the device
                p.kill()
                p.join(timeout=30)
        assert p.exitcode == 0, (name, p.exitcode)
    a = res["local"]
    assert res["rccl_graphs"]["captures"] >= 1 and res["rccl_eager"]["captures"] == 0
    assert res["rccl_graphs"]["backend"] == "nccl"
    for name in ("rccl_eager", "rccl_graphs"):
        b = res[name]
        assert a["losses"] == b["losses"], name
        for k in ("E", "w", "m", "v"):
            if a[k] is not None:
                assert np.array_equal(a[k], b[k]), (name, k)
        for k in a["dense"]:
            assert np.array_equal(a["dense"][k], b["dense"][k]), (name, k)
