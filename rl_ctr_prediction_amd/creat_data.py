"""libsvm_dataset — the reference's map-style dataset (src/models/creat_data.py:3-19).

Rows of ``label,idx_1..idx_F`` as produced by src/encode/data_.py:85; the default collate
gives int64 [B,F] features and int64 [B] labels.
"""
from __future__ import annotations

import torch.utils.data as data


class libsvm_dataset(data.Dataset):  # noqa: N801 (reference name)
    def __init__(self, Data, label):
        super().__init__()
        self.Data = Data
        self.label = label

    def __len__(self):
        return len(self.Data)

    def __getitem__(self, item):
        return self.Data[item], self.label[item]
