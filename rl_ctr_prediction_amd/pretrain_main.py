"""CTR pretraining driver — counterpart of ``src/all_main/pretrain_main.py``.

Same functions (setup_seed, get_model, get_dataset, train, test, submission, main,
eva_stopping), same flags and files (train_.txt / test_.txt / featindex.txt in, rotating
``{model}{epoch%5}.pth`` + ``{model}best.pth`` + ``test_submission.csv`` / ``day_aucs.csv``
out), same semantics: batches in file order (no shuffle), Adam re-created every epoch
(here: :meth:`FusedCTRTrainer.reset_optimizer`), train loss = mean of batch losses,
AUC over the concatenated test predictions, loss-/AUC-based early stopping with reload
of the checkpoint four epochs back.

Differences, all deliberate: the training step is the fused HIP step (FM, DeepFM and
IPNN; FFM: FusedFFMTrainer, the same deferred-exact Adam over its F*V field-table rows;
AutogradTrainer keeps the autograd + torch.optim.Adam route for comparison; the other six model families are out of scope); the batches are
sliced from one device-resident copy of the data instead of 8 DataLoader worker
processes; the rotating-checkpoint cleanup skips files that were never written (the
reference crashes there when epoch < 5, all_main/pretrain_main.py:201-202).
"""
from __future__ import annotations

import argparse
import datetime
import os
import random

import numpy as np
import pandas as pd
import torch
import torch.nn as nn
from sklearn.metrics import roc_auc_score

from . import creat_data as Data
from .binfmt import load_encoded
from . import p_model as Model
from .ffm_trainer import FusedFFMTrainer
from .trainer import FusedCTRTrainer


def setup_seed(seed):
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)
    random.seed(seed)


def get_model(model_name, feature_nums, field_nums, latent_dims):
    if model_name == "FM":
        return Model.FM(feature_nums, latent_dims)
    if model_name == "DeepFM":
        return Model.DeepFM(feature_nums, field_nums, latent_dims)
    if model_name == "IPNN":
        return Model.InnerPNN(feature_nums, field_nums, latent_dims)
    if model_name == "FFM":
        return Model.FFM(feature_nums, field_nums, latent_dims)
    raise NotImplementedError(
        f"{model_name}: FM, FFM, DeepFM and IPNN are built on HIP; "
        "LR/W&D/FNN/OPNN/DCN/AFM are out of scope (SURVEY.md §2 row 7)")


class AutogradTrainer:
    """The reference's own step (all_main/pretrain_main.py:72-79: forward, BCELoss,
    zero_grad, backward, torch.optim.Adam.step) through autograd (tests compare it with the
    fused trainers): the
    forward / backward run on the HIP kernels through autograd, the dense gradients go to
    an unchanged torch.optim.Adam, re-created every epoch like the reference (line 153)."""

    def __init__(self, model, lr, weight_decay):
        self.model, self.lr, self.weight_decay = model, lr, weight_decay
        self.loss = nn.BCELoss()
        self.reset_optimizer()

    def reset_optimizer(self, lr=None):
        if lr is not None:
            self.lr = lr
        self.opt = torch.optim.Adam(self.model.parameters(), lr=self.lr,
                                    weight_decay=self.weight_decay)

    def step(self, features, labels):
        y = self.model(features)
        loss = self.loss(y, labels.view(-1, 1).float())
        self.model.zero_grad()
        loss.backward()
        self.opt.step()
        return loss.detach()

    def check_errors(self):
        pass


def get_dataset(datapath, dataset_name, campaign_id, binary=True):
    """binary: read train_/test_ through their CTRBIN01 sidecars (rl_ctr_prediction_amd.binfmt:
    converted once by the native parser, memory-mapped afterwards) instead of pd.read_csv —
    the same integer matrix."""
    data_path = datapath + dataset_name + campaign_id
    if binary:
        train_fm = load_encoded(data_path + "train_.txt")
        test_fm = load_encoded(data_path + "test_.txt")
    else:
        train_fm = pd.read_csv(data_path + "train_.txt", header=None).values.astype(int)
        test_fm = pd.read_csv(data_path + "test_.txt", header=None).values.astype(int)
    field_nums = len(train_fm[0, 1:])
    feature_index = pd.read_csv(data_path + "featindex.txt", header=None).values
    feature_nums = int(feature_index[-1, 0].split("\t")[1]) + 1
    return train_fm, train_fm, test_fm, field_nums, feature_nums


class DeviceBatches:
    """Batches of a libsvm_dataset in file order, sliced from one device-resident copy
    (features int64 [N,F] like the reference's collated LongTensor, labels float)."""

    def __init__(self, dataset: Data.libsvm_dataset, batch_size: int, device):
        # np.array copies: the data may be a read-only memory map (binfmt.open_bin)
        self.x = torch.from_numpy(np.array(dataset.Data, dtype=np.int64)).to(device)
        self.y = torch.from_numpy(np.array(dataset.label, dtype=np.float32)).to(device)
        self.batch_size = int(batch_size)

    def __len__(self):
        return (self.x.shape[0] + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        for s in range(0, self.x.shape[0], self.batch_size):
            yield self.x[s:s + self.batch_size], self.y[s:s + self.batch_size]


def train(model, optimizer, data_loader, loss, device):
    """One epoch (all_main/pretrain_main.py:67-83); `optimizer` is the fused trainer.

    The reference reads every batch loss on the host (``total_loss += train_loss.item()``,
    line 79): a full sync per step. The fused trainers add each step's loss to a float64
    accumulator on the device inside the step's last launch, and the epoch reads it once —
    the same fp32 values added in the same order in double: bitwise the reference's Python
    float sum (tests/test_gpu_models.py::test_driver_epoch_loss_bitwise)."""
    model.train()
    batches = list(data_loader)  # views of the device-resident data: nothing is copied
    return run_epoch(optimizer, batches)


def run_epoch(optimizer, batches) -> float:
    """Mean train loss of one pass of `optimizer` over `batches` [(features, labels)] in
    order (the body of train(); bench.py --driver-loop times it)."""
    if not batches:
        raise ZeroDivisionError("float division by zero")  # the reference's empty epoch
    lookahead = isinstance(optimizer, FusedCTRTrainer)
    device_sum = hasattr(optimizer, "read_loss_sum")
    total_loss = 0.0
    if device_sum:
        optimizer.reset_loss_sum()
    for i, (features, labels) in enumerate(batches):
        if lookahead:  # the next two batches' sparse plans are built during this step
            nxt = batches[i + 1:i + 3]
            optimizer.step(features, labels, next_x=[b[0] for b in nxt], return_loss=False,
                           next_y=[b[1] for b in nxt])
        elif device_sum:
            optimizer.step(features, labels, return_loss=False)
        else:  # AutogradTrainer: the reference's per-step host read
            total_loss += optimizer.step(features, labels).item()
    if device_sum:
        total_loss = optimizer.read_loss_sum()
    optimizer.check_errors()
    return total_loss / len(batches)


def _predict(model, data_loader, loss):
    model.eval()
    targets, predicts = [], []
    intervals, total = 0, 0.0
    with torch.no_grad():
        for features, labels in data_loader:
            y = model(features)
            total += loss(y, labels.view(-1, 1)).item()
            targets.extend(labels.view(-1, 1).tolist())
            predicts.extend(y.tolist())
            intervals += 1
    return targets, predicts, total / max(intervals, 1)


def test(model, data_loader, loss, device):
    targets, predicts, avg = _predict(model, data_loader, loss)
    return roc_auc_score(targets, predicts), avg


def submission(model, data_loader, device):
    targets, predicts, _ = _predict(model, data_loader, nn.BCELoss())
    return predicts, roc_auc_score(targets, predicts)


def eva_stopping(valid_aucs, valid_losses, type):  # noqa: A002 (reference name)
    if type == "auc":
        if len(valid_aucs) >= 5:
            a = valid_aucs
            if a[-1] < a[-2] < a[-3] < a[-4] < a[-5]:
                return True
    else:
        if len(valid_losses) >= 5:
            v = valid_losses
            if v[-1] > v[-2] > v[-3] > v[-4] > v[-5]:
                return True
    return False


def main(data_path, dataset_name, campaign_id, latent_dims, model_name, epoch, learning_rate,
         weight_decay, early_stop_type, batch_size, device, save_param_dir, verbose=True,
         _epoch_fn=None):
    """_epoch_fn(model, trainer, train_fm, loss, device, batch_size) -> mean train loss: the
    epoch loop of a driver variant (pretrain_main_2's slicing loop); default: DeviceBatches."""
    if not os.path.exists(save_param_dir + campaign_id):
        os.mkdir(save_param_dir + campaign_id)
    device = torch.device(device)
    train_fm, train_data, test_data, field_nums, feature_nums = get_dataset(
        data_path, dataset_name, campaign_id)
    test_dataset = Data.libsvm_dataset(test_data[:, 1:], test_data[:, 0])
    test_data_loader = DeviceBatches(test_dataset, batch_size, device)
    if _epoch_fn is None:
        train_dataset = Data.libsvm_dataset(train_data[:, 1:], train_data[:, 0])
        train_data_loader = DeviceBatches(train_dataset, batch_size, device)

    model = get_model(model_name, feature_nums, field_nums, latent_dims).to(device)
    loss = nn.BCELoss()
    if model_name == "FFM":
        trainer = FusedFFMTrainer(model, lr=learning_rate, weight_decay=weight_decay)
    else:
        trainer = FusedCTRTrainer(model, lr=learning_rate, weight_decay=weight_decay)

    valid_aucs, valid_losses, history = [], [], []
    early_stop_index, is_early_stop = 0, False
    start_time = datetime.datetime.now()
    for epoch_i in range(epoch):
        train_start_time = datetime.datetime.now()
        trainer.reset_optimizer()  # torch.optim.Adam(...) re-created every epoch (line 153)
        if _epoch_fn is None:
            train_average_loss = train(model, trainer, train_data_loader, loss, device)
        else:
            train_average_loss = _epoch_fn(model, trainer, train_fm, loss, device, batch_size)
        torch.save(model.state_dict(),
                   save_param_dir + campaign_id + model_name + str(np.mod(epoch_i, 5)) + ".pth")
        auc, valid_loss = test(model, test_data_loader, loss, device)
        valid_aucs.append(auc)
        valid_losses.append(valid_loss)
        history.append(dict(epoch=epoch_i, train_loss=train_average_loss, valid_auc=auc,
                            valid_loss=valid_loss))
        train_end_time = datetime.datetime.now()
        if verbose:
            print("epoch:", epoch_i, "training average loss:", train_average_loss,
                  "validation auc:", auc, "validation loss:", valid_loss,
                  "[{}s]".format((train_end_time - train_start_time).seconds))
        if eva_stopping(valid_aucs, valid_losses, early_stop_type):
            early_stop_index = np.mod(epoch_i - 4, 5)
            is_early_stop = True
            break
    end_time = datetime.datetime.now()

    if is_early_stop:
        test_model = get_model(model_name, feature_nums, field_nums, latent_dims).to(device)
        load_path = save_param_dir + campaign_id + model_name + str(early_stop_index) + ".pth"
        test_model.load_state_dict(torch.load(load_path, map_location=device, weights_only=True))
    else:
        test_model = model
    auc, test_loss = test(test_model, test_data_loader, loss, device)
    torch.save(test_model.state_dict(), save_param_dir + campaign_id + model_name + "best.pth")
    if verbose:
        print("\ntest auc:", auc, datetime.datetime.now(),
              "[{}s]".format((end_time - start_time).seconds))

    submission_path = data_path + dataset_name + campaign_id + model_name + "/"
    if not os.path.exists(submission_path):
        os.mkdir(submission_path)
    test_predicts, test_auc = submission(test_model, test_data_loader, device)
    pd.DataFrame(data=test_predicts).to_csv(submission_path + "test_submission.csv", header=None)
    pd.DataFrame(data=[[test_auc]]).to_csv(submission_path + "day_aucs.csv", header=None)
    for i in range(5):
        path = save_param_dir + campaign_id + model_name + str(i) + ".pth"
        if os.path.exists(path):
            os.remove(path)
    return dict(history=history, test_auc=auc, test_loss=test_loss, test_preds=test_predicts,
                model=test_model)


def _parser():
    parser = argparse.ArgumentParser()
    parser.add_argument("--data_path", default="../../data/")
    parser.add_argument("--dataset_name", default="avazu/", help="ipinyou, cretio, yoyi, avazu")
    parser.add_argument("--campaign_id", default="avazu/", help="1458, 3358, 3386, 3427, 3476, avazu")
    parser.add_argument("--model_name", default="FM", help="FM, FFM, DeepFM, IPNN")
    parser.add_argument("--latent_dims", type=int, default=10)
    parser.add_argument("--epoch", type=int, default=20)
    parser.add_argument("--learning_rate", type=float, default=1e-3)
    parser.add_argument("--weight_decay", type=float, default=1e-5)
    parser.add_argument("--early_stop_type", default="loss", help="auc, loss")
    parser.add_argument("--batch_size", type=int, default=4096)
    parser.add_argument("--device", default="cuda:0")
    parser.add_argument("--save_param_dir", default="../models/model_params/")
    return parser


if __name__ == "__main__":
    args = _parser().parse_args()
    setup_seed(1)
    main(args.data_path, args.dataset_name, args.campaign_id, args.latent_dims, args.model_name,
         args.epoch, args.learning_rate, args.weight_decay, args.early_stop_type,
         args.batch_size, args.device, args.save_param_dir)
