"""CTR pretraining driver, day-split variant — counterpart of ``src/main/pretrain_main.py``.

What differs from the ``all_main`` driver (rl_ctr_prediction_amd/pretrain_main.py), as in the
reference:
  * the data is ONE encoded file ``train.txt`` plus ``day_index.csv`` rows (day, first row,
    last row); one day is the validation set, one the test set, the other days (in
    day_index order) the training set; ``feature_nums`` = the largest id + 1
    (main/pretrain_main.py:47-88);
  * ``learning_rate += 1e-4`` before every epoch's fresh Adam (:180-181) — here
    ``FusedCTRTrainer.reset_optimizer(lr=...)``, which rewrites the per-step Adam scalars in
    place (captured HIP graphs keep running);
  * early stopping watches the validation day; the test day is scored at the end, and
    both days' predictions and AUCs are written (``{day}_test_submission.csv``,
    ``day_aucs.csv`` rows [day, auc]) (:206-238);
  * IPNN / FNN / OPNN start from the FM-pretrained embedding
    ``models/model_params/{campaign}FMbest.pth`` (:166-168; FNN/OPNN are out of scope).

Same flags and defaults as the reference (:256-269). The training step is the fused HIP
step; batches come in file order from one device-resident copy (the reference's
DataLoader without shuffle).
"""
from __future__ import annotations

import argparse
import datetime
import os

import numpy as np
import pandas as pd
import torch
import torch.nn as nn

from .. import creat_data as Data
from ..ffm_trainer import FusedFFMTrainer
from ..pretrain_main import (DeviceBatches, eva_stopping, get_model, setup_seed,
                             submission, test, train)
from ..trainer import FusedCTRTrainer

__all__ = ["setup_seed", "get_model", "get_dataset", "train", "test", "submission", "main",
           "eva_stopping"]


def get_dataset(datapath, dataset_name, campaign_id, valid_day, test_day):
    """(train_fm, day_indexs, train_data, valid_data, test_data, field_nums, feature_nums)
    as main/pretrain_main.py:47-88 builds them."""
    data_path = datapath + dataset_name + campaign_id
    train_fm = pd.read_csv(data_path + "train.txt", header=None).values.astype(int)
    field_nums = len(train_fm[0, 1:])
    feature_nums = int(np.max(train_fm[:, 1:].flatten())) + 1
    day_indexs = pd.read_csv(data_path + "day_index.csv", header=None).values
    days = day_indexs[:, 0]
    days_list = days.tolist()
    days_list.pop(days_list.index(valid_day))
    days_list.pop(days_list.index(test_day))

    def rows_of(day):
        d = day_indexs[days == day]
        return train_fm[d[0, 1]: d[0, 2] + 1, :]

    train_data = np.concatenate([rows_of(day) for day in days_list], axis=0)
    return (train_fm, day_indexs, train_data, rows_of(valid_day), rows_of(test_day), field_nums,
            feature_nums)


def main(data_path, dataset_name, campaign_id, valid_day, test_day, latent_dims, model_name, epoch,
         learning_rate, weight_decay, early_stop_type, batch_size, device, save_param_dir,
         verbose=True):
    if not os.path.exists(save_param_dir + campaign_id):
        os.mkdir(save_param_dir + campaign_id)
    device = torch.device(device)
    _, _, train_data, valid_data, test_data, field_nums, feature_nums = get_dataset(
        data_path, dataset_name, campaign_id, valid_day, test_day)
    loaders = [DeviceBatches(Data.libsvm_dataset(d[:, 1:], d[:, 0]), batch_size, device)
               for d in (train_data, valid_data, test_data)]
    train_data_loader, valid_data_loader, test_data_loader = loaders

    model = get_model(model_name, feature_nums, field_nums, latent_dims).to(device)
    if model_name == "IPNN":  # main/pretrain_main.py:166-168
        fm_params = torch.load("models/model_params/" + campaign_id + "FMbest.pth",
                               map_location=device, weights_only=True)
        model.load_embedding(fm_params)
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
        learning_rate += 1e-4  # main/pretrain_main.py:180
        trainer.reset_optimizer(lr=learning_rate)
        train_average_loss = train(model, trainer, train_data_loader, loss, device)
        torch.save(model.state_dict(),
                   save_param_dir + campaign_id + model_name + str(np.mod(epoch_i, 5)) + ".pth")
        auc, valid_loss = test(model, valid_data_loader, loss, device)
        valid_aucs.append(auc)
        valid_losses.append(valid_loss)
        history.append(dict(epoch=epoch_i, lr=learning_rate, train_loss=train_average_loss,
                            valid_auc=auc, valid_loss=valid_loss))
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
    valid_predicts, valid_auc = submission(test_model, valid_data_loader, device)
    pd.DataFrame(data=valid_predicts).to_csv(
        submission_path + str(valid_day) + "_test_submission.csv", header=None)
    test_predicts, test_auc = submission(test_model, test_data_loader, device)
    pd.DataFrame(data=test_predicts).to_csv(
        submission_path + str(test_day) + "_test_submission.csv", header=None)
    pd.DataFrame(data=[[valid_day, valid_auc], [test_day, test_auc]]).to_csv(
        submission_path + "day_aucs.csv", header=None)
    for i in range(5):
        path = save_param_dir + campaign_id + model_name + str(i) + ".pth"
        if os.path.exists(path):  # (the reference crashes here when epoch < 5)
            os.remove(path)
    return dict(history=history, test_auc=auc, test_loss=test_loss, valid_preds=valid_predicts,
                test_preds=test_predicts, valid_auc=valid_auc, model=test_model)


def _parser():
    parser = argparse.ArgumentParser()
    parser.add_argument("--data_path", default="../../data/")
    parser.add_argument("--dataset_name", default="ipinyou/", help="ipinyou, creti o, yoyi")
    parser.add_argument("--valid_day", type=int, default=11, help="6, 7, 8, 9, 10, 11, 12")
    parser.add_argument("--test_day", type=int, default=12, help="6, 7, 8, 9, 10, 11, 12")
    parser.add_argument("--campaign_id", default="1458/", help="1458, 3358, 3386, 3427, 3476")
    parser.add_argument("--model_name", default="FM", help="FM, FFM, DeepFM, IPNN")
    parser.add_argument("--latent_dims", type=int, default=8)
    parser.add_argument("--epoch", type=int, default=100)
    parser.add_argument("--learning_rate", type=float, default=1e-4)
    parser.add_argument("--weight_decay", type=float, default=1e-5)
    parser.add_argument("--early_stop_type", default="loss", help="auc, loss")
    parser.add_argument("--batch_size", type=int, default=2048)
    parser.add_argument("--device", default="cuda:0")
    parser.add_argument("--save_param_dir", default="../models/model_params/")
    return parser


if __name__ == "__main__":
    args = _parser().parse_args()
    setup_seed(1)
    main(args.data_path, args.dataset_name, args.campaign_id, args.valid_day, args.test_day,
         args.latent_dims, args.model_name, args.epoch, args.learning_rate, args.weight_decay,
         args.early_stop_type, args.batch_size, args.device, args.save_param_dir)
