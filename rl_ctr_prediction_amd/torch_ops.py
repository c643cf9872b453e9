"""The PyTorch op layer of the drop-in boundary: the ABI kernels registered
as ``torch.library`` custom ops in namespace ``ctr``, each differentiable one with its
autograd formula and every one with a fake (meta) kernel for shape propagation.

    torch.ops.ctr.fm_fwd(x, emb, lin, bias) -> (z [B,1], sum_e [B,K])
        FM logit, p_model.FM.forward (p_model.py:40-57) minus the sigmoid; sum_e = the
        per-example field sums sum_f E[x_f] (kept for the backward; not differentiable).
        Backward: ctr::fm_bwd.
    torch.ops.ctr.fm_bwd(x, emb, sum_e, gz) -> (g_emb [V,K], g_lin [V,1], g_bias [1])
        the dense gradients embedding_dense_backward + the bias sum would produce (rows
        summed in slot order, deterministic).
    torch.ops.ctr.deepfm_gather_concat(x, emb) -> flat [B, F*K]
        DeepFM's MLP input, the second gather of p_model.py:320. Backward: ctr::emb_scatter_add.
    torch.ops.ctr.emb_scatter_add(x, grad_slots [B*F,K], num_rows) -> dense [num_rows,K]
        embedding_dense_backward: G[r] = sum of the slot gradients of row r, in slot order.
    torch.ops.ctr.ipnn_cat(x, emb) -> [B, F*K + F(F-1)/2]
        InnerPNN's MLP input (p_model.py:187-195). Backward: per-slot gradients, then
        ctr::emb_scatter_add.
    torch.ops.ctr.pairwise_fe(x, emb) -> [B, F(F-1)/2 + F*K]
        Feature_Embedding.forward (Feature_embedding.py:51-59); the reference detaches the
        result, so no autograd formula (pass a detached table, as Feature_Embedding does).
    torch.ops.ctr.adam_dense(p!, g, m!, v!, step, lr, beta1, beta2, eps, weight_decay)
        one torch.optim.Adam step (coupled L2) on a dense parameter (all_main/pretrain_main.py:78).
    torch.ops.ctr.adam_rowwise(emb!, m!, v!, rows, grad_rows, step, lr, beta1, beta2, eps,
                               weight_decay)
        the same step on a [V,K] table whose gradient is grad_rows[u] at row rows[u] (rows
        unique) and zero elsewhere — every row still moves (weight decay, momentum), as the
        reference's dense Adam does.
    torch.ops.ctr.pg_returns(r, gamma) -> (vt fp64, vt fp32)
        PolicyGradient.discount_and_norm_rewards (PG_model.py:139-154).

Inputs must be ROCm tensors (the ops refuse CPU tensors: there is no CPU fallback).
Indices may be int64 (what the reference hands) or int32.
"""
from __future__ import annotations

import torch
from torch import Tensor

from . import hip_ops

__all__ = ["fm_fwd", "fm_bwd", "deepfm_gather_concat", "emb_scatter_add", "ipnn_cat",
           "pairwise_fe", "adam_dense", "adam_rowwise", "pg_returns"]

_lib = torch.library


def _f32(*shape, like: Tensor) -> Tensor:
    return like.new_empty(shape, dtype=torch.float32)


def _scatter_dense(x: Tensor, grad_slots: Tensor, num_rows: int) -> Tensor:
    S = x.numel()
    K = grad_slots.shape[-1]
    vals = grad_slots.reshape(S, K).contiguous()
    plan = hip_ops.SparsePlanBuffers(S, vals.device).build(x.reshape(-1), num_rows)
    rows, _ = hip_ops.segment_sum_rows(plan, vals)
    return hip_ops.rows_to_dense(plan, num_rows, rows)[0]


# ------------------------------------------------------------------------- FM (A1) ----
@_lib.custom_op("ctr::fm_fwd", mutates_args=())
def fm_fwd(x: Tensor, emb: Tensor, lin: Tensor, bias: Tensor) -> tuple[Tensor, Tensor]:
    B = x.shape[0]
    r = hip_ops.fm_forward(x, emb, lin, bias, want_sum=True, want_p=False)
    return r.z.view(B, 1), r.sum_e


@fm_fwd.register_fake
def _(x, emb, lin, bias):
    return _f32(x.shape[0], 1, like=emb), _f32(x.shape[0], emb.shape[1], like=emb)


@_lib.custom_op("ctr::fm_bwd", mutates_args=())
def fm_bwd(x: Tensor, emb: Tensor, sum_e: Tensor, gz: Tensor) -> tuple[Tensor, Tensor, Tensor]:
    B, F = x.shape
    V, _ = emb.shape
    gz = gz.reshape(-1).contiguous()
    plan = hip_ops.SparsePlanBuffers(B * F, emb.device).build(x, V)
    rows, rows_lin = hip_ops.fm_embedding_grad(plan, F, emb, gz, sum_e)
    g_emb, g_lin = hip_ops.rows_to_dense(plan, V, rows, rows_lin)
    return g_emb, g_lin, hip_ops.tensor_sum(gz).view(1)


@fm_bwd.register_fake
def _(x, emb, sum_e, gz):
    V, K = emb.shape
    return _f32(V, K, like=emb), _f32(V, 1, like=emb), _f32(1, like=emb)


def _fm_setup(ctx, inputs, output):
    x, emb, _, _ = inputs
    ctx.mark_non_differentiable(output[1])
    ctx.save_for_backward(x, emb, output[1])


def _fm_backward(ctx, gz, _gsum):
    x, emb, sum_e = ctx.saved_tensors
    if gz is None:
        gz = torch.zeros(x.shape[0], 1, dtype=torch.float32, device=emb.device)
    g_emb, g_lin, g_bias = torch.ops.ctr.fm_bwd(x, emb, sum_e, gz)
    return None, g_emb, g_lin, g_bias


fm_fwd.register_autograd(_fm_backward, setup_context=_fm_setup)


# ------------------------------------------------------------ gather / scatter (A3) ----
@_lib.custom_op("ctr::emb_scatter_add", mutates_args=())
def emb_scatter_add(x: Tensor, grad_slots: Tensor, num_rows: int) -> Tensor:
    return _scatter_dense(x, grad_slots, num_rows)


@emb_scatter_add.register_fake
def _(x, grad_slots, num_rows):
    return _f32(num_rows, grad_slots.shape[-1], like=grad_slots)


@_lib.custom_op("ctr::deepfm_gather_concat", mutates_args=())
def deepfm_gather_concat(x: Tensor, emb: Tensor) -> Tensor:
    B, F = x.shape
    return hip_ops.embedding_gather(emb, x).view(B, F * emb.shape[1])


@deepfm_gather_concat.register_fake
def _(x, emb):
    return _f32(x.shape[0], x.shape[1] * emb.shape[1], like=emb)


def _gather_setup(ctx, inputs, output):
    x, emb = inputs
    ctx.save_for_backward(x)
    ctx.V = emb.shape[0]


def _gather_backward(ctx, gflat):
    (x,) = ctx.saved_tensors
    B, F = x.shape
    g = gflat.reshape(B * F, -1).contiguous()
    return None, torch.ops.ctr.emb_scatter_add(x, g, ctx.V)


deepfm_gather_concat.register_autograd(_gather_backward, setup_context=_gather_setup)


# ------------------------------------------------------------- IPNN (§8f rank 1) ----
@_lib.custom_op("ctr::ipnn_cat", mutates_args=())
def ipnn_cat(x: Tensor, emb: Tensor) -> Tensor:
    return hip_ops.ipnn_forward(x, emb)


@ipnn_cat.register_fake
def _(x, emb):
    F = x.shape[1]
    return _f32(x.shape[0], F * emb.shape[1] + F * (F - 1) // 2, like=emb)


def _ipnn_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _ipnn_backward(ctx, gcat):
    x, emb = ctx.saved_tensors
    dslot = hip_ops.ipnn_backward(x, emb, gcat.contiguous())
    return None, torch.ops.ctr.emb_scatter_add(x, dslot, emb.shape[0])


ipnn_cat.register_autograd(_ipnn_backward, setup_context=_ipnn_setup)


# ----------------------------------------------------------- Feature_Embedding (A7) ----
@_lib.custom_op("ctr::pairwise_fe", mutates_args=())
def pairwise_fe(x: Tensor, emb: Tensor) -> Tensor:
    return hip_ops.feature_embedding(x, emb)


@pairwise_fe.register_fake
def _(x, emb):
    F = x.shape[1]
    return _f32(x.shape[0], F * (F - 1) // 2 + F * emb.shape[1], like=emb)


# ------------------------------------------------------------------------ Adam (A5) ----
@_lib.custom_op("ctr::adam_dense", mutates_args=("p", "m", "v"))
def adam_dense(p: Tensor, g: Tensor, m: Tensor, v: Tensor, step: int, lr: float, beta1: float,
               beta2: float, eps: float, weight_decay: float) -> None:
    hip_ops.adam_dense(p, g.contiguous(), m, v, step, lr, (beta1, beta2), eps, weight_decay)


@adam_dense.register_fake
def _(p, g, m, v, step, lr, beta1, beta2, eps, weight_decay):
    return None


@_lib.custom_op("ctr::adam_rowwise", mutates_args=("emb", "m", "v"))
def adam_rowwise(emb: Tensor, m: Tensor, v: Tensor, rows: Tensor, grad_rows: Tensor, step: int,
                 lr: float, beta1: float, beta2: float, eps: float, weight_decay: float) -> None:
    V, K = emb.shape
    n = rows.numel()
    if grad_rows.shape != (n, K):
        raise ValueError(f"adam_rowwise: grad_rows must be [{n}, {K}], got {tuple(grad_rows.shape)}")
    rowmap = torch.full((V,), -1, dtype=torch.int32, device=emb.device)
    rowmap.index_copy_(0, rows.reshape(-1).long(),
                       torch.arange(n, dtype=torch.int32, device=emb.device))
    hip_ops.adam_embedding(emb, m, v, None, None, None, rowmap, grad_rows.contiguous(), None,
                           step, lr, (beta1, beta2), eps, weight_decay)


@adam_rowwise.register_fake
def _(emb, m, v, rows, grad_rows, step, lr, beta1, beta2, eps, weight_decay):
    return None


# ------------------------------------------------------------ REINFORCE returns (A8) ----
@_lib.custom_op("ctr::pg_returns", mutates_args=())
def pg_returns(r: Tensor, gamma: float) -> tuple[Tensor, Tensor]:
    vt, vt32, _ = hip_ops.pg_discount_norm(r, gamma)
    return vt, vt32


@pg_returns.register_fake
def _(r, gamma):
    n = r.numel()
    return r.new_empty(n, dtype=torch.float64), r.new_empty(n, dtype=torch.float32)
