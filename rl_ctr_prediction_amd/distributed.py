"""Data-parallel exchange for the CTR step: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on ROCm; "gloo" for the CPU tests).

Examples are independent and the loss is a mean, so the global-batch gradient is a sum
of per-rank gradients computed with the GLOBAL mean divisor:
  * dense parameters (FM bias, DeepFM MLP: 0.56 M floats) live in one flat buffer ->
    ONE all-reduce per step (latency-bound at 2.2 MB; a single bucket is optimal);
  * embedding gradients are exchanged sparsely: each rank all-gathers every rank's
    (unique row, row-sum) pairs and re-sums them by row in (rank, row) order with the
    deterministic segmented sum, so every replica applies bit-identical dense Adam and
    the replicated tables never diverge — no V x K all-reduce (2.6 GB at C3).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def allreduce_sum_(t: torch.Tensor, group=None, force: bool = False) -> torch.Tensor:
    """In-place sum over the group's ranks. force: issue the collective at world size 1 too
    (a one-rank RCCL communicator: the N > 1 launch sequence exercised on one GPU)."""
    if world()[1] > 1 or force:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def allgather_sparse_rows(rows: torch.Tensor, vals: torch.Tensor, lin: torch.Tensor | None,
                          count: int, group=None):
    """Concatenate every rank's first `count` (rows, vals, lin) entries in rank order.

    rows [>=count] int32, vals [>=count, K] fp32, lin [>=count] fp32 (optional). Counts
    differ per rank, so the payload is padded to the largest count for the collective
    and the padding is dropped on receipt. Returns (rows_all, vals_all, lin_all).
    """
    rank, ws = world()
    if ws == 1:
        return rows[:count], vals[:count], None if lin is None else lin[:count]
    dev = rows.device
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(ws)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    cap = max(max(counts), 1)
    K = vals.shape[1]
    width = K + 1 if lin is not None else K  # [vals | lin]
    send_rows = torch.zeros(cap, dtype=torch.int32, device=dev)
    send_rows[:count] = rows[:count].to(torch.int32)
    send = torch.zeros(cap, width, dtype=torch.float32, device=dev)
    send[:count, :K] = vals[:count]
    if lin is not None:
        send[:count, K] = lin[:count]
    recv_rows = torch.empty(ws * cap, dtype=torch.int32, device=dev)
    recv = torch.empty(ws * cap, width, dtype=torch.float32, device=dev)
    dist.all_gather_into_tensor(recv_rows, send_rows, group=group)
    dist.all_gather_into_tensor(recv, send, group=group)
    recv_rows = recv_rows.view(ws, cap)
    recv = recv.view(ws, cap, width)
    rows_all = torch.cat([recv_rows[r, :counts[r]] for r in range(ws)]).contiguous()
    allp = torch.cat([recv[r, :counts[r]] for r in range(ws)], dim=0)
    vals_all = allp[:, :K].contiguous()
    lin_all = allp[:, K].contiguous() if lin is not None else None
    return rows_all, vals_all, lin_all


def allgather_varlen(t: torch.Tensor, group=None) -> tuple[torch.Tensor, list[int]]:
    """Concatenation, in rank order, of every rank's 1-D tensor `t` (lengths may differ)
    -> (the concatenation, per-rank lengths). Padded to the longest for the collective."""
    rank, ws = world()
    n = t.numel()
    if ws == 1:
        return t.reshape(-1), [n]
    stage = t.is_cuda and dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if stage else t.device
    cnt = torch.tensor([n], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(ws)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    cap = max(max(counts), 1)
    send = torch.zeros(cap, dtype=t.dtype, device=dev)
    send[:n] = t.reshape(-1).to(dev)
    recv = torch.empty(ws * cap, dtype=t.dtype, device=dev)
    dist.all_gather_into_tensor(recv, send, group=group)
    recv = recv.view(ws, cap)
    out = torch.cat([recv[r, :counts[r]] for r in range(ws)]).to(t.device)
    return out, counts


def alltoallv(send: torch.Tensor, send_counts: list[int], recv_counts: list[int],
              group=None) -> torch.Tensor:
    """Variable-split all-to-all along dim 0: rank r sends send[sum(send_counts[:j]) ...]
    (send_counts[j] rows) to rank j and receives recv_counts[j] rows from rank j, in rank
    order. RCCL (nccl backend) moves device tensors directly over xGMI; the gloo backend
    (CPU test runs) stages device tensors through host memory."""
    rank, ws = world()
    out = torch.empty((sum(recv_counts),) + tuple(send.shape[1:]), dtype=send.dtype,
                      device=send.device)
    if ws == 1:
        out.copy_(send[:recv_counts[0]])
        return out
    n = sum(send_counts)
    src = send[:n].contiguous()
    if send.is_cuda and dist.get_backend(group) == "gloo":
        o = out.cpu()
        dist.all_to_all_single(o, src.cpu(), recv_counts, send_counts, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, src, recv_counts, send_counts, group=group)
    return out


def alltoall_equal(out: torch.Tensor, send: torch.Tensor, group=None,
                   force: bool = False) -> torch.Tensor:
    """Equal-split all-to-all along dim 0 (N equal blocks of the same rows each way): sizes
    fixed by the shapes, no host-side counts — the row-sharded exchange at a fixed capacity.
    One process: a copy, unless force (the collective on a one-rank communicator). gloo (CPU
    test runs) stages device tensors through host memory."""
    rank, ws = world()
    if ws == 1 and not force:
        out.copy_(send)
        return out
    if send.is_cuda and dist.get_backend(group) == "gloo":
        o = out.cpu()
        dist.all_to_all_single(o, send.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, send, group=group)
    return out


def exchange_counts(counts: torch.Tensor, group=None) -> tuple[list[int], list[int]]:
    """counts[j] = rows this rank sends to rank j (int64 device tensor) -> (send_counts,
    recv_counts) host lists. One small all-to-all and one host sync per call: the
    variable-split collectives need the sizes on the host."""
    rank, ws = world()
    if ws == 1:
        c = counts.tolist()
        return c, c
    recv = alltoallv(counts.view(ws, 1), [1] * ws, [1] * ws, group).view(-1)
    return counts.tolist(), recv.tolist()
