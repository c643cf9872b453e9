"""Feature_Embedding on the HIP pairwise kernel — drop-in for
``src/models/Feature_embedding.py:31-59`` (the RL state encoder).

forward(x [B,F]) -> [B, F(F-1)/2 + F*K] = [<E[x_i],E[x_j]> for i<j (row-major pair
order, lines 40-43)] ++ flat(E[x]); detached, like the reference (line 59).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import hip_ops


class Feature_Embedding(nn.Module):  # noqa: N801 (reference name)
    def __init__(self, feature_numbers, field_nums, latent_dims):
        super().__init__()
        self.field_nums = field_nums
        self.latent_dims = int(latent_dims)
        self.feature_embedding = nn.Embedding(feature_numbers, self.latent_dims)
        self.row, self.col = [], []
        for i in range(self.field_nums - 1):
            for j in range(i + 1, self.field_nums):
                self.row.append(i)
                self.col.append(j)

    def load_embedding(self, pretrain_params):
        """Copy a pretrained FM table (Feature_embedding.py:45-49)."""
        self.feature_embedding.weight.data.copy_(
            torch.from_numpy(np.array(pretrain_params["feature_embedding.weight"].cpu())))

    def forward(self, x):
        return hip_ops.feature_embedding(x, self.feature_embedding.weight.detach())
