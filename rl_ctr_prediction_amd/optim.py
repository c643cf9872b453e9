"""``DenseAdam``: torch.optim.Adam (coupled L2, the reference's optimizer,
all_main/pretrain_main.py:78,153) on the ABI's Adam kernel — the optimizer half of the op
layer (SURVEY.md §8b ``ctr.optim.DenseAdam``), for models trained through autograd on the
HIP ops (dense gradients, e.g. ``p_model.FM`` / ``FFM`` or ``torch.ops.ctr.*`` compositions).

Same constructor, same ``param_groups`` and the same ``state`` keys as torch.optim.Adam
(``step``, ``exp_avg``, ``exp_avg_sq``), so checkpoints move between the two. Every element
moves every step (weight decay and momentum on rows without gradient), as the reference's
dense Adam does. The per-step scalars lr/(1-beta1^t) and 1/sqrt(1-beta2^t) are formed in
Python doubles and rounded once, as torch does; each parameter is one ``ctr_adam_dense``
launch (csrc/adam.hip ``adam_elem``, the arithmetic every fused trainer path shares).
"""
from __future__ import annotations

import torch

from . import hip_ops


class DenseAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False):
        if amsgrad:
            raise NotImplementedError("DenseAdam: amsgrad (the reference never uses it)")
        if lr < 0.0 or eps < 0.0 or weight_decay < 0.0:
            raise ValueError("DenseAdam: lr, eps and weight_decay must be >= 0")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"DenseAdam: invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay, amsgrad=False))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, betas = group["lr"], group["betas"]
            eps, wd = group["eps"], group["weight_decay"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("DenseAdam: sparse gradients are not supported")
                if not p.is_contiguous():
                    raise RuntimeError("DenseAdam: parameters must be contiguous")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] += 1
                t = int(st["step"].item())
                hip_ops.adam_dense(p.view(-1), p.grad.contiguous().view(-1),
                                   st["exp_avg"].view(-1), st["exp_avg_sq"].view(-1), t, lr,
                                   betas, eps, wd)
        return loss
