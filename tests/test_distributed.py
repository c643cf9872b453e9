"""Data-parallel exchange on CPU with gloo, world size 2 (the N>1 path's host logic).

Each rank builds the per-row gradient sums of its own batch (the oracle's numpy
grouping stands in for the GPU scatter kernel), exchanges them with
allgather_sparse_rows, re-sums by row in (rank, row) order and must obtain the
gradient of the GLOBAL batch — identical on both ranks. The dense flat buffer goes
through one all-reduce.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import collect_ranks


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _row_sums(keys, vals, lin):
    uniq, inv = np.unique(keys, return_inverse=True)
    out = np.zeros((uniq.size, vals.shape[1]), np.float64)
    outl = np.zeros(uniq.size, np.float64)
    np.add.at(out, inv, vals)
    np.add.at(outl, inv, lin)
    return uniq, out, outl


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rl_ctr_prediction_amd.distributed import allgather_sparse_rows, allreduce_sum_, world as w
        assert w() == (rank, world)
        rng = np.random.default_rng(100 + rank)
        K = 8
        n = 300 + 57 * rank                      # ragged: ranks hold different row counts
        keys = rng.integers(0, 120, size=n)
        vals = rng.standard_normal((n, K))
        lin = rng.standard_normal(n)
        uniq, rs, rl = _row_sums(keys, vals, lin)
        cap = uniq.size + 5                      # buffers larger than the valid count
        rows_t = torch.zeros(cap, dtype=torch.int32)
        rows_t[: uniq.size] = torch.tensor(uniq, dtype=torch.int32)
        vals_t = torch.zeros(cap, K)
        vals_t[: uniq.size] = torch.tensor(rs, dtype=torch.float32)
        lin_t = torch.zeros(cap)
        lin_t[: uniq.size] = torch.tensor(rl, dtype=torch.float32)
        r_all, v_all, l_all = allgather_sparse_rows(rows_t, vals_t, lin_t, uniq.size)
        g_uniq, g_sum, g_lin = _row_sums(r_all.numpy(), v_all.numpy().astype(np.float64),
                                         l_all.numpy().astype(np.float64))
        flat = torch.full((1000,), float(rank + 1))
        allreduce_sum_(flat)
        q.put((rank, g_uniq, g_sum, g_lin, r_all.numpy(), float(flat[0])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_sparse_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for r in collect_ranks(procs, q, world):
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # expected: the global batch's per-row sums
    keys, vals, lin = [], [], []
    for rank in range(world):
        rng = np.random.default_rng(100 + rank)
        n = 300 + 57 * rank
        keys.append(rng.integers(0, 120, size=n))
        vals.append(rng.standard_normal((n, 8)))
        lin.append(rng.standard_normal(n))
    gu, gs, gl = _row_sums(np.concatenate(keys), np.concatenate(vals), np.concatenate(lin))
    for rank in range(world):
        u, s, l_, rows_all, flat0 = res[rank]
        np.testing.assert_array_equal(u, gu)
        np.testing.assert_allclose(s, gs, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(l_, gl, rtol=1e-5, atol=1e-5)
        assert flat0 == world * (world + 1) / 2  # sum of rank + 1
    # every rank received the same concatenation (rank order), so the re-sums agree bitwise
    for rank in range(1, world):
        np.testing.assert_array_equal(res[0][3], res[rank][3])
        np.testing.assert_array_equal(res[0][1], res[rank][1])


# ------------------------------------------------------------ row-sharded exchange ----
def _shard_worker(rank, world, port, q):
    """The ShardedCTRTrainer protocol with numpy standing in for the GPU kernels (plan,
    shard counts, gather, segmented sum): ids to owners, rows back, gradients to owners."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rl_ctr_prediction_amd.distributed import alltoallv, exchange_counts
        V, K = 1000, 4
        shard = -(-V // world)
        lo, hi = rank * shard, min(V, (rank + 1) * shard)
        table = np.arange(V * K, dtype=np.float32).reshape(V, K)   # the same on every rank
        rng = np.random.default_rng(7 + rank)
        ids = rng.integers(0, V, size=500 + 111 * rank)
        ids[:50] = 3                                               # a hot row on every rank
        uniq = np.unique(ids)                                      # the plan's unique rows
        counts = np.array([((uniq >= j * shard) & (uniq < (j + 1) * shard)).sum()
                           for j in range(world)], dtype=np.int64)  # ctr_plan_shard_counts
        send_c, recv_c = exchange_counts(torch.tensor(counts))
        req = alltoallv(torch.tensor(uniq, dtype=torch.int32), send_c, recv_c)
        loc = req.numpy() - lo
        assert ((loc >= 0) & (loc < hi - lo)).all()                # every request is mine
        rows = torch.tensor(table[lo:hi][loc])                     # owner gathers its rows
        got = alltoallv(rows, recv_c, send_c).numpy()
        np.testing.assert_array_equal(got, table[uniq])            # rows back in unique order
        # per-row gradient of this rank: count of the row in the batch x (rank + 1)
        cnt = np.array([(ids == u).sum() for u in uniq], dtype=np.float32)
        grads = torch.tensor(np.repeat((cnt * (rank + 1))[:, None], K, axis=1))
        G = alltoallv(grads, send_c, recv_c).numpy()
        keys = req.numpy()
        u_o = np.unique(keys)
        sums = np.stack([G[keys == u].sum(0) for u in u_o]) if u_o.size else np.zeros((0, K))
        q.put((rank, u_o, sums))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [3, 8])
def test_row_sharded_exchange_gloo(world):
    """The row-sharded protocol at world sizes 3 and 8 (the target node: 8 x MI355X)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for r in collect_ranks(procs, q, world):
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    V, K = 1000, 4
    shard = -(-V // world)
    expect = np.zeros(V)
    for rank in range(world):
        rng = np.random.default_rng(7 + rank)
        ids = rng.integers(0, V, size=500 + 111 * rank)
        ids[:50] = 3
        np.add.at(expect, ids, rank + 1)
    for rank in range(world):
        u_o, sums = res[rank]
        assert ((u_o >= rank * shard) & (u_o < (rank + 1) * shard)).all()
        np.testing.assert_array_equal(u_o, np.nonzero(expect[rank * shard:(rank + 1) * shard])[0]
                                      + rank * shard)
        np.testing.assert_allclose(sums[:, 0], expect[u_o])


# ------------------------------------------------- fixed-capacity (padded) exchange ----
def _padded_worker(rank, world, port, q, layout="blocks"):
    """ShardedCTRTrainer's fixed-capacity protocol with numpy standing in for the GPU
    kernels (ctr_shard_permute_ids / ctr_shard_pack_ids_layout / ctr_shard_runs_copy):
    capacity agreed by an all-reduce MAX, equal-split all-to-alls of ids, rows and gradients,
    padding entries on each owner's spare row (index = its row count). layout "cyclic": rank r
    owns the rows r::N, the ids permuted to (r % N) * Vs + r // N before the plan, so each
    owner's unique rows are again one ascending run."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rl_ctr_prediction_amd.distributed import alltoall_equal
        V, K = 1000, 4
        shard = -(-V // world)
        cyc = layout == "cyclic"
        table = np.arange(V * K, dtype=np.float32).reshape(V, K)
        own = table[rank::world] if cyc else table[rank * shard:min(V, (rank + 1) * shard)]
        n_own = own.shape[0]
        mine = np.concatenate([own, np.full((1, K), -7, np.float32)])  # + spare row
        rng = np.random.default_rng(7 + rank)
        ids = rng.integers(0, V, size=500 + 111 * rank)
        ids[:50] = 3
        keys = (ids % world) * shard + ids // world if cyc else ids
        uniq = np.unique(keys)
        orig = (uniq % shard) * world + uniq // shard if cyc else uniq  # back to global rows
        owner = uniq // shard
        counts = np.bincount(owner, minlength=world)
        offsets = np.concatenate([[0], np.cumsum(counts)[:-1]])
        cap = torch.tensor([int(counts.max())])
        dist.all_reduce(cap, op=dist.ReduceOp.MAX)
        C = int(-(-int(cap) // 64) * 64)
        send = np.empty(world * C, np.int32)
        for j in range(world):
            spare = len(range(j, V, world)) if cyc else min(shard, V - j * shard)
            run = uniq[offsets[j]:offsets[j] + counts[j]] - j * shard
            send[j * C:(j + 1) * C] = np.concatenate([run, np.full(C - counts[j], spare)])
        recv = torch.empty(world * C, dtype=torch.int32)
        alltoall_equal(recv, torch.tensor(send))
        loc = recv.numpy()
        assert ((loc >= 0) & (loc <= n_own)).all()
        rows_in = torch.empty(world * C, K)
        alltoall_equal(rows_in, torch.tensor(mine[loc]))
        got = np.concatenate([rows_in.numpy()[j * C:j * C + counts[j]] for j in range(world)])
        np.testing.assert_array_equal(got, table[orig])          # unpacked, compact order
        cnt = np.array([(ids == u).sum() for u in orig], dtype=np.float32)
        g = np.repeat((cnt * (rank + 1))[:, None], K, axis=1)
        g_pad = np.zeros((world * C, K), np.float32)
        for j in range(world):
            g_pad[j * C:j * C + counts[j]] = g[offsets[j]:offsets[j] + counts[j]]
        g_in = torch.empty(world * C, K)
        alltoall_equal(g_in, torch.tensor(g_pad))
        sums = np.zeros((n_own + 1, K), np.float32)
        np.add.at(sums, loc, g_in.numpy())
        assert (sums[-1] == 0).all()                               # padding: zero gradients
        nz = np.nonzero(sums[:-1, 0])[0]
        rows = nz * world + rank if cyc else nz + rank * shard     # local -> global rows
        q.put((rank, rows, sums[nz]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,layout", [(2, "blocks"), (5, "blocks"), (3, "cyclic"),
                                          (8, "cyclic")])
def test_padded_exchange_gloo(world, layout):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_padded_worker, args=(r, world, port, q, layout))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in collect_ranks(procs, q, world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    V = 1000
    shard = -(-V // world)
    expect = np.zeros(V)
    for rank in range(world):
        rng = np.random.default_rng(7 + rank)
        ids = rng.integers(0, V, size=500 + 111 * rank)
        ids[:50] = 3
        np.add.at(expect, ids, rank + 1)
    for rank in range(world):
        rows, sums = res[rank]
        if layout == "cyclic":
            mine = np.arange(rank, V, world)
            want = mine[expect[mine] != 0]
        else:
            want = np.nonzero(expect[rank * shard:(rank + 1) * shard])[0] + rank * shard
        np.testing.assert_array_equal(rows, want)
        np.testing.assert_allclose(sums[:, 0], expect[rows])
