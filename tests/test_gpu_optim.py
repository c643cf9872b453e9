"""DenseAdam (rl_ctr_prediction_amd/optim.py, SURVEY §8b ``ctr.optim.DenseAdam``): the
reference's training loop (all_main/pretrain_main.py:72-79: forward, BCELoss, zero_grad,
backward, optimizer.step) with torch.optim.Adam swapped for DenseAdam, against the
reference's own two Adam steps (g_deepfm.npz, g_ffm.npz), and its state_dict against
torch.optim.Adam's."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import AdamBound, assert_grad_close

pytestmark = pytest.mark.gpu


def _model(g, kind, dev):
    import rl_ctr_prediction_amd as P
    keys = [str(k) for k in g["keys"]] if "keys" in g.files else None
    if kind == "DeepFM":
        V, K = g["init/feature_embedding.weight"].shape
        F = g["init/mlp.0.weight"].shape[1] // K
        m = P.DeepFM(V, F, K).to(dev)
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0  # the goldens' protocol (dropout is RNG-dependent)
        keys = [k for k in m.state_dict()]
    else:
        V, K = g["init/field_feature_embeddings.0.weight"].shape
        F = sum(k.startswith("field_feature_embeddings.") for k in keys)
        m = P.FFM(V, F, K).to(dev)
    m.load_state_dict({k: torch.tensor(g[f"init/{k}"]) for k in keys})
    return m, keys


@pytest.mark.parametrize("kind,name", [("DeepFM", "g_deepfm.npz"), ("FFM", "g_ffm.npz")])
def test_dense_adam_two_steps_vs_reference(cuda, golden, kind, name):
    from rl_ctr_prediction_amd.optim import DenseAdam
    g = golden(name)
    m, keys = _model(g, kind, cuda)
    opt = DenseAdam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    bd = {k: AdamBound(g[f"init/{k}"], 1e-3, 1e-5) for k in keys}
    for s in range(2):
        x, y = torch.tensor(g[f"x{s}"], device=cuda), torch.tensor(g[f"y{s}"], device=cuda)
        loss = torch.nn.BCELoss()(m(x), y.view(-1, 1))
        assert loss.item() == pytest.approx(float(g[f"loss{s}"]), rel=1e-5)
        opt.zero_grad()
        loss.backward()
        named = dict(m.named_parameters())
        tol = {k: assert_grad_close(named[k].grad.cpu().numpy(), g[f"grad{s}/{k}"],
                                    err_msg=f"grad {k}") for k in keys}
        opt.step()
        sd = m.state_dict()
        for k in keys:
            bd[k].step(g[f"grad{s}/{k}"], tol[k]).check(sd[k].cpu().numpy(),
                                                       g[f"step{s + 1}/{k}"], err_msg=k)


def test_dense_adam_state_dict_round_trips_with_torch_adam(cuda):
    """DenseAdam's state_dict loads into torch.optim.Adam and back (same keys and shapes),
    and the first moment follows torch's lerp exactly on a fixed gradient."""
    from rl_ctr_prediction_amd.optim import DenseAdam
    torch.manual_seed(3)
    p1 = torch.nn.Parameter(torch.randn(300, 16, device=cuda) * 0.1)
    p2 = torch.nn.Parameter(p1.detach().clone())
    a = DenseAdam([p1], lr=1e-3, weight_decay=1e-5)
    b = torch.optim.Adam([p2], lr=1e-3, weight_decay=1e-5, foreach=False)
    g = torch.randn(300, 16, device=cuda) * 1e-3
    for _ in range(3):
        p1.grad, p2.grad = g.clone(), g.clone()
        a.step()
        b.step()
    sa, sb = a.state_dict(), b.state_dict()
    assert sa["param_groups"][0]["lr"] == sb["param_groups"][0]["lr"]
    assert set(sa["state"][0]) >= {"step", "exp_avg", "exp_avg_sq"}
    assert float(sa["state"][0]["step"]) == float(sb["state"][0]["step"]) == 3.0
    # parameters within a few ulps of the step (Adam's sqrt / division are not
    # correctly rounded in either implementation)
    np.testing.assert_allclose(p1.detach().cpu().numpy(), p2.detach().cpu().numpy(),
                               rtol=1e-6, atol=1e-9)
    c = torch.optim.Adam([p1], lr=1e-3, weight_decay=1e-5)
    c.load_state_dict(sa)
    d = DenseAdam([p2], lr=1e-3, weight_decay=1e-5)
    d.load_state_dict(sb)
    assert float(d.state_dict()["state"][0]["step"]) == 3.0
    p2.grad = g.clone()
    d.step()  # continues from torch's moments
    assert float(d.state_dict()["state"][0]["step"]) == 4.0
