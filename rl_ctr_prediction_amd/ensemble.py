"""`generate_preds` of the RL drivers on one HIP kernel.

Drop-in for ``generate_preds(model_dict, features, actions, prob_weights, c_actions, labels,
device, mode)`` (``src/all_main/hybrid_td3_main_per_v10.py:54-164``; the same function in
the other hybrid_* drivers): the M frozen CTR models' pCTRs, then the per-example ensemble
(top-``action`` models by ``prob_weights``, softmax weights of the top ``c_actions``), the
±1/0 sign reward against the models' mean, and the returned continuous actions — the
reference's per-action Python loop of masks, sorts and scatters becomes one rank pass and
one thread-per-example kernel (csrc/ensemble.hip: ``ctr_ensemble_preds``). Semantics kept
exactly, including the reference's indexing of ``sort_c_actions`` with action-group-local
positions (line 127).
"""
from __future__ import annotations

import torch

from . import hip_ops


def generate_preds(model_dict, features, actions, prob_weights, c_actions, labels, device,
                   mode=None):
    """Returns (y_preds [B,1], rewards [B,1], return_c_actions [B,M]) like the reference."""
    M = len(model_dict)
    with torch.no_grad():
        preds = torch.cat([model_dict[i](features).detach().reshape(-1, 1).float()
                           for i in range(M)], dim=1).contiguous()
    return hip_ops.ensemble_preds(preds, actions.to(device), prob_weights.float().to(device),
                                  c_actions.float().to(device), labels.to(device))
