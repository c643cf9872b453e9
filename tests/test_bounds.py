"""The parity bars themselves (conftest.AdamBound / grad_bound), on the CPU: torch.optim.Adam
fed gradients anywhere inside the bar stays inside the interval, and a parameter moved by
a fraction of one step where the gradient is large falls outside."""
from __future__ import annotations

import numpy as np
import torch

from conftest import AdamBound, grad_bound


def _run(p0, grads, lr, wd):
    p = torch.tensor(p0, dtype=torch.float32, requires_grad=True)
    opt = torch.optim.Adam([p], lr=lr, weight_decay=wd)
    for g in grads:
        p.grad = torch.tensor(g, dtype=torch.float32)
        opt.step()
    return p.detach().numpy()


def test_adam_bound_contains_every_gradient_inside_the_bar():
    rng = np.random.default_rng(0)
    n, steps, lr, wd = 20000, 3, 1e-3, 1e-5
    p0 = rng.normal(0, 0.05, n).astype(np.float32)
    # magnitudes from 1e-12 (|g| << eps: the steep region) to 1
    grads = [(rng.normal(size=n) * 10.0 ** rng.uniform(-12, 0, n)).astype(np.float32)
             for _ in range(steps)]
    bd = AdamBound(p0, lr, wd)
    tols = []
    for g in grads:
        tols.append(grad_bound(g))
        bd.step(g, tols[-1])
    ref = _run(p0, grads, lr, wd)
    bd.check(ref, err_msg="unperturbed")
    for trial in range(4):  # gradients perturbed anywhere inside (and at the edge of) the bar
        pert = [(g + t * rng.choice([-1.0, 1.0, rng.uniform(-1, 1)], size=n)).astype(np.float32)
                for g, t in zip(grads, tols)]
        bd.check(_run(p0, pert, lr, wd), ref, err_msg=f"trial {trial}")


def test_adam_bound_rejects_a_wrong_step():
    rng = np.random.default_rng(1)
    n, lr = 1000, 1e-3
    p0 = rng.normal(0, 0.05, n).astype(np.float32)
    g = rng.normal(0, 1e-2, n).astype(np.float32)  # |g| >> eps: the step is ~lr exactly
    bd = AdamBound(p0, lr, 0.0).step(g, grad_bound(g))
    ref = _run(p0, [g], lr, 0.0)
    bd.check(ref)
    bad = ref.copy()
    bad[17] += 0.01 * lr  # 1 % of one Adam step on one element
    try:
        bd.check(bad)
    except AssertionError as e:
        assert "1/1000" in str(e)
    else:
        raise AssertionError("a 1 % step error went unnoticed")
