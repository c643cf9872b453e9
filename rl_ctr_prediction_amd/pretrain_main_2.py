"""CTR pretraining driver, preloaded-tensor variant — counterpart of
``src/all_main/pretrain_main_2.py``.

The reference's variant of all_main/pretrain_main.py keeps the encoded training matrix as
ONE LongTensor and slices batches out of it, ``train_data[i:i+batch, 1:]`` /
``train_data[i:i+batch, 0]`` for i in range(0, len_train, batch) (pretrain_main_2.py:61,
67-72), instead of a DataLoader over a libsvm_dataset. Here the LongTensor is
device-resident and each slice is a view fed to the fused HIP step; everything else
(files, early stopping, Adam re-created per epoch, outputs) is the all_main driver's.
"""
from __future__ import annotations

import numpy as np
import torch

from . import pretrain_main as _pm
from .pretrain_main import (eva_stopping, get_model, setup_seed, submission,  # noqa: F401
                            test, _parser)

__all__ = ["setup_seed", "get_model", "get_dataset", "train", "test", "submission", "main",
           "eva_stopping"]


def get_dataset(datapath, dataset_name, campaign_id):
    """(train_fm, train_data LongTensor [N, 1+F], test_data, field_nums, feature_nums)
    (pretrain_main_2.py:47-62)."""
    train_fm, _, test_fm, field_nums, feature_nums = _pm.get_dataset(datapath, dataset_name,
                                                                     campaign_id)
    # copied first: train_fm may be a read-only memory map of the binary batch cache
    return (train_fm, torch.from_numpy(np.array(train_fm, dtype=np.int64)), test_fm, field_nums,
            feature_nums)


def train(model, optimizer, train_data, loss, device, len_train, batch):
    """One epoch over slices of the preloaded tensor (pretrain_main_2.py:64-79);
    `optimizer` is the fused trainer, `train_data` the [N, 1+F] LongTensor (moved to the
    device once)."""
    model.train()
    data = train_data.to(device)
    batches = [(data[i:i + batch, 1:], data[i:i + batch, 0].float())
               for i in range(0, len_train, batch)]
    return _pm.run_epoch(optimizer, batches)  # the loss summed on the device, read once


def main(data_path, dataset_name, campaign_id, latent_dims, model_name, epoch, learning_rate,
         weight_decay, early_stop_type, batch_size, device, save_param_dir, verbose=True):
    cache = {}

    def epoch_fn(model, trainer, train_fm, loss, dev, bs):
        if "data" not in cache:  # the LongTensor of get_dataset, moved once
            # copied first: a read-only memory map is not handed to torch as it is
            cache["data"] = torch.from_numpy(np.array(train_fm, dtype=np.int64)).to(dev)
        return train(model, trainer, cache["data"], loss, dev, len(train_fm), bs)

    return _pm.main(data_path, dataset_name, campaign_id, latent_dims, model_name, epoch,
                    learning_rate, weight_decay, early_stop_type, batch_size, device,
                    save_param_dir, verbose=verbose, _epoch_fn=epoch_fn)


if __name__ == "__main__":
    args = _parser().parse_args()
    setup_seed(1)
    main(args.data_path, args.dataset_name, args.campaign_id, args.latent_dims, args.model_name,
         args.epoch, args.learning_rate, args.weight_decay, args.early_stop_type,
         args.batch_size, args.device, args.save_param_dir)
