"""Data-parallel REINFORCE (C4) on the GPU: two ranks (gloo, one GPU) each
holding half of an episode must learn what one process learns from the whole episode.

The returns, their mean and every per-sample logit gradient are bit-identical by
construction (pg_model.PolicyGradient.learn); the weight gradients are the two halves'
sums added by the all-reduce — another association order than one GEMM over the whole
episode — so parameters are held to the Adam bar. The loss (loss_func = mean(nlp * vt))
is nlp times the mean of NORMALISED returns, i.e. times their rounding residue: one
process sums the n terms nlp*vt_b (|nlp| ~ n ln A ~ 400 here), whose rounding alone is
~u*nlp*mean|vt| ~ 2e-5 absolute, while the ranks form nlp_r*mean(vt) — so the loss value
is cancellation noise in BOTH (the single-process values are 0 or +-1.5e-5) and its bar
is absolute, 4*u*nlp.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import collect_ranks, AdamBound, grad_bound

pytestmark = pytest.mark.gpu

V, F, K, A, N_EP, EPISODES = 500, 6, 4, 5, 256, 3


def _episodes(seed=5):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(EPISODES):
        x = torch.randint(0, V, (N_EP, F), generator=g)
        a = torch.randint(1, A + 1, (N_EP, 1), generator=g)
        r = torch.randn(N_EP, 1, generator=g)
        out.append((x, a, r))
    return out


def _agent(train: bool):
    import rl_ctr_prediction_amd as P
    torch.manual_seed(7)
    pg = P.PolicyGradient(V, F, K, "dp", action_nums=A, device="cuda:0", fix_input_dims=True)
    pg.policy_net.train(train)
    return pg


def _learn(pg, episodes, lo, hi, grads=None):
    losses = []
    for x, a, r in episodes:
        pg.store_transition(x[lo:hi].cuda(), a[lo:hi].cuda(), r[lo:hi].cuda())
        losses.append(float(pg.learn().item()))
        if grads is not None:  # the episode's (all-reduced) MLP gradient
            grads.append([g.detach().cpu().numpy().copy() for g in pg._gviews])
    return losses


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, train, cuts, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        pg = _agent(train)
        p0 = {k: v.detach().cpu().numpy().copy() for k, v in pg.policy_net.mlp.state_dict().items()}
        grads = []
        losses = _learn(pg, _episodes(), cuts[rank], cuts[rank + 1], grads)
        params = {k: v.detach().cpu().numpy() for k, v in pg.policy_net.mlp.state_dict().items()}
        q.put((rank, losses, params, p0, grads, pg.lr, pg.weight_decay))
    finally:
        dist.destroy_process_group()


def _run(world, train, cuts):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, train, cuts, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for r in collect_ranks(procs, q, world):
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("train,cuts", [(False, (0, 128, 256)), (True, (0, 100, 256))])
def test_pg_dp_world2_matches_whole_episode(cuda, train, cuts):
    # the single-process reference also runs in a fresh process: the dropout seed is
    # drawn from a per-process counter (p_model._dropout_seed), as in the ranks
    ref_losses, ref, p0, ref_grads, lr, wd = _run(1, train, (0, N_EP))[0]
    res = _run(2, train, cuts)
    nlp = N_EP * np.log(A)
    # per-element Adam interval from the one-process run's per-episode gradients and the
    # gradient bar (1e-5*|g| + 1e-6*max|g|) assumed for the ranks' all-reduced gradients
    bd = {k: AdamBound(v, lr, wd) for k, v in p0.items()}
    for step in ref_grads:
        for k, g in zip(p0, step):
            bd[k].step(g, grad_bound(g))
    for rank in range(2):
        losses, params = res[rank][:2]
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-5, atol=4 * 2.0**-24 * nlp)
        for k, v in params.items():
            bd[k].check(v, ref[k], err_msg=f"{k} rank {rank}")
    for k in res[0][1]:  # replicas stay bit-identical
        assert np.array_equal(res[0][1][k], res[1][1][k]), k
