"""Capture golden vectors from the reference implementation (survey container only).

Imports jqsl2012/RL_CTR_Prediction from /root/reference (read-only, never copied) and
runs it on CPU to produce small input/output fixtures in this directory. The fixtures are
data: inputs, initial parameters and the reference's outputs. The GPU box never sees the
reference; tests there compare against these files.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [fixture ...]

(no argument: every fixture; else only the named ones, e.g. `ipnn`)

Fixtures:
  g_fm.npz       FM fwd/bwd + 2 Adam steps (std 0.1 init) and an N(0,1) saturated case
  g_deepfm.npz   DeepFM fwd/bwd + 2 Adam steps, dropout p=0 (train mode)
  g_ipnn.npz     InnerPNN fwd/bwd + 2 Adam steps, dropout p=0 (train mode)
  g_ffm.npz      FFM fwd/bwd + 2 Adam steps (std 0.1 tables)
  g_ensemble.npz generate_preds of the RL drivers (hybrid_td3_main_per_v10.py:54-164) on
                 fixed pretrained-model pCTRs (stand-in models returning them)
  g_bce.npz      sigmoid + BCELoss values and d/dz incl. saturated logits
  g_fe.npz       Feature_Embedding forward
  g_pg.npz       PolicyGradient: discount_and_norm_rewards, loss_func (+ grads), choose_action
  toy/           C1 toy data (13 dense bucketised + 26 sparse fields, 1000 rows)
  g_toy.json     pretrain_main.main on the toy (FM, FFM, and DeepFM / IPNN with dropout p=0):
                 per-epoch train loss / valid AUC / valid loss, final test AUC and preds
  toy_days/ + g_toy_days.json  src/main/pretrain_main.py on the toy split into days 6..12
                 (valid 11, test 12; lr += 1e-4 per epoch): FM, DeepFM
  g_toy_2.json   src/all_main/pretrain_main_2.py (preloaded-tensor slicing) on the toy
  manifest.json  versions and seeds
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import re
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REF = Path(os.environ.get("CTR_REFERENCE", "/root/reference"))


def _import_reference():
    if not REF.exists():
        raise SystemExit(f"{REF} not found: goldens are generated in the survey container only")
    sys.dont_write_bytecode = True
    sys.path.insert(0, str(REF))
    import src.models.p_model as P  # noqa: E402
    import src.models.Feature_embedding as FE  # noqa: E402
    import src.models.PG_model as PG  # noqa: E402
    import src.all_main.pretrain_main as PM  # noqa: E402
    return P, FE, PG, PM


def _np(t):
    return t.detach().cpu().numpy().copy()


def _hot_ids(g, B, F, V):
    x = torch.randint(0, V, (B, F), generator=g)
    x[:, 0] = 7                              # one row owning B slots (spans many chunks)
    x[: B // 2, 1] = 3                       # two rows sharing a field
    x[B // 2:, 1] = 4
    x[:, 2] = x[:, 3]                        # duplicates inside an example
    return x


def gen_fm(P):
    out = {}
    V, F, K, B = 1000, 26, 16, 64
    for tag, std in (("small", 0.1), ("sat", None)):
        torch.manual_seed(0)
        m = P.FM(V, K)
        with torch.no_grad():
            if std is not None:
                m.feature_embedding.weight.normal_(0, std)
                m.linear.weight.normal_(0, std)
                m.bias.fill_(0.05)
        g = torch.Generator().manual_seed(1)
        xs = [_hot_ids(g, B, F, V) for _ in range(2)]
        ys = [(torch.rand(B, 1, generator=g) < 0.3).float() for _ in range(2)]
        out[f"{tag}_E0"] = _np(m.feature_embedding.weight)
        out[f"{tag}_w0"] = _np(m.linear.weight)
        out[f"{tag}_b0"] = _np(m.bias)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
        crit = torch.nn.BCELoss()
        for s in range(2):
            x, y = xs[s], ys[s]
            p = m(x)
            loss = crit(p, y)
            m.zero_grad()
            loss.backward()
            out[f"{tag}_x{s}"] = _np(x)
            out[f"{tag}_y{s}"] = _np(y)
            out[f"{tag}_p{s}"] = _np(p)
            out[f"{tag}_loss{s}"] = np.float32(loss.item())
            out[f"{tag}_gE{s}"] = _np(m.feature_embedding.weight.grad)
            out[f"{tag}_gw{s}"] = _np(m.linear.weight.grad)
            out[f"{tag}_gb{s}"] = _np(m.bias.grad)
            opt.step()
            out[f"{tag}_E{s + 1}"] = _np(m.feature_embedding.weight)
            out[f"{tag}_w{s + 1}"] = _np(m.linear.weight)
            out[f"{tag}_b{s + 1}"] = _np(m.bias)
    np.savez(HERE / "g_fm.npz", **out)


DEEPFM_KEYS = ["bias", "linear.weight", "feature_embedding.weight", "mlp.0.weight", "mlp.0.bias",
               "mlp.3.weight", "mlp.3.bias", "mlp.6.weight", "mlp.6.bias"]


def gen_deepfm(P):
    out = {}
    V, F, K, B = 500, 8, 16, 64
    torch.manual_seed(0)
    m = P.DeepFM(V, F, K)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    with torch.no_grad():
        m.feature_embedding.weight.normal_(0, 0.1)
        m.linear.weight.normal_(0, 0.1)
        m.bias.fill_(-0.1)
    sd = m.state_dict()
    for k in DEEPFM_KEYS:
        out[f"init/{k}"] = _np(sd[k])
    g = torch.Generator().manual_seed(2)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    crit = torch.nn.BCELoss()
    m.train()
    for s in range(2):
        x = _hot_ids(g, B, F, V)
        y = (torch.rand(B, 1, generator=g) < 0.3).float()
        p = m(x)
        loss = crit(p, y)
        m.zero_grad()
        loss.backward()
        out[f"x{s}"] = _np(x)
        out[f"y{s}"] = _np(y)
        out[f"p{s}"] = _np(p)
        out[f"loss{s}"] = np.float32(loss.item())
        named = dict(m.named_parameters())
        for k in DEEPFM_KEYS:
            out[f"grad{s}/{k}"] = _np(named[k].grad)
        opt.step()
        sd = m.state_dict()
        for k in DEEPFM_KEYS:
            out[f"step{s + 1}/{k}"] = _np(sd[k])
    np.savez(HERE / "g_deepfm.npz", **out)


IPNN_KEYS = ["feature_embedding.weight", "mlp.0.weight", "mlp.0.bias", "mlp.3.weight",
             "mlp.3.bias", "mlp.6.weight", "mlp.6.bias"]


def gen_ipnn(P):
    """InnerPNN (p_model.py:146-200): same protocol as gen_deepfm; std 0.1 embeddings."""
    out = {}
    V, F, K, B = 500, 8, 16, 64
    torch.manual_seed(0)
    m = P.InnerPNN(V, F, K)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    with torch.no_grad():
        m.feature_embedding.weight.normal_(0, 0.1)
    sd = m.state_dict()
    for k in IPNN_KEYS:
        out[f"init/{k}"] = _np(sd[k])
    g = torch.Generator().manual_seed(3)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    crit = torch.nn.BCELoss()
    m.train()
    for s in range(2):
        x = _hot_ids(g, B, F, V)
        y = (torch.rand(B, 1, generator=g) < 0.3).float()
        p = m(x)
        loss = crit(p, y)
        m.zero_grad()
        loss.backward()
        out[f"x{s}"] = _np(x)
        out[f"y{s}"] = _np(y)
        out[f"p{s}"] = _np(p)
        out[f"loss{s}"] = np.float32(loss.item())
        named = dict(m.named_parameters())
        for k in IPNN_KEYS:
            out[f"grad{s}/{k}"] = _np(named[k].grad)
        opt.step()
        sd = m.state_dict()
        for k in IPNN_KEYS:
            out[f"step{s + 1}/{k}"] = _np(sd[k])
    np.savez(HERE / "g_ipnn.npz", **out)


def gen_ffm(P):
    """FFM (p_model.py:59-100): same protocol as gen_deepfm."""
    out = {}
    V, F, K, B = 300, 6, 8, 64
    torch.manual_seed(0)
    m = P.FFM(V, F, K)
    with torch.no_grad():
        for e in m.field_feature_embeddings:
            e.weight.normal_(0, 0.1)
        m.linear.weight.normal_(0, 0.1)
        m.bias.fill_(-0.1)
    keys = list(m.state_dict().keys())
    out["keys"] = np.array(keys)
    sd = m.state_dict()
    for k in keys:
        out[f"init/{k}"] = _np(sd[k])
    g = torch.Generator().manual_seed(4)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5)
    crit = torch.nn.BCELoss()
    for s in range(2):
        x = _hot_ids(g, B, F, V)
        y = (torch.rand(B, 1, generator=g) < 0.3).float()
        p = m(x)
        loss = crit(p, y)
        m.zero_grad()
        loss.backward()
        out[f"x{s}"] = _np(x)
        out[f"y{s}"] = _np(y)
        out[f"p{s}"] = _np(p)
        out[f"loss{s}"] = np.float32(loss.item())
        named = dict(m.named_parameters())
        for k in keys:
            out[f"grad{s}/{k}"] = _np(named[k].grad)
        opt.step()
        sd = m.state_dict()
        for k in keys:
            out[f"step{s + 1}/{k}"] = _np(sd[k])
    np.savez(HERE / "g_ffm.npz", **out)


def gen_ensemble():
    """The reference's generate_preds with M stand-in models that return fixed pCTR columns
    (the function only calls model_dict[i](features).detach())."""
    import src.all_main.hybrid_td3_main_per_v10 as H  # noqa: E402
    out = {}
    g = torch.Generator().manual_seed(7)
    for case, (B, M) in enumerate([(257, 5), (64, 3), (1500, 8), (40, 1)]):
        preds = torch.rand(B, M, generator=g)
        model_dict = {i: (lambda x, i=i: preds[:, i:i + 1]) for i in range(M)}
        feats = torch.zeros(B, 2, dtype=torch.long)
        actions = torch.randint(1, M + 1, (B, 1), generator=g)
        pw = torch.softmax(torch.randn(B, M, generator=g), dim=1)
        ca = torch.rand(B, M, generator=g) * 2 - 1
        labels = torch.randint(0, 2, (B, 1), generator=g)
        y, r, rc = H.generate_preds(model_dict, feats, actions, pw, ca, labels, "cpu", "train")
        for k, v in dict(preds=preds, actions=actions, pw=pw, ca=ca, labels=labels, y=y, r=r,
                         rc=rc).items():
            out[f"c{case}_{k}"] = _np(v)
    np.savez(HERE / "g_ensemble.npz", **out)


def gen_bce():
    z = torch.tensor([0.0, 0.3, -0.3, 2.0, -2.0, 8.0, -8.0, 15.0, -15.0, 16.5, -16.5, 17.0, -17.0,
                      30.0, -30.0, 50.0, -50.0, 88.0, -88.0, 90.0, -90.0, 104.0, -104.0, 1e-4,
                      -1e-4, 5.5, -5.5, 12.25, 40.0, -40.0, 103.0, -103.5], dtype=torch.float32)
    g = torch.Generator().manual_seed(3)
    z = torch.cat([z, torch.randn(96, generator=g) * 20])
    y = (torch.rand(z.numel(), generator=g) < 0.4).float()
    y[:32:2] = 1.0
    y[1:32:2] = 0.0
    zz = z.clone().requires_grad_(True)
    p = torch.sigmoid(zz)
    loss = torch.nn.BCELoss()(p, y)
    loss.backward()
    np.savez(HERE / "g_bce.npz", z=_np(z), y=_np(y), p=_np(p), loss=np.float32(loss.item()),
             gz=_np(zz.grad))


def gen_fe(FE):
    V, F, K, B = 1000, 26, 16, 32
    torch.manual_seed(5)
    fe = FE.Feature_Embedding(V, F, K)
    g = torch.Generator().manual_seed(6)
    x = _hot_ids(g, B, F, V)
    out = fe(x)
    np.savez(HERE / "g_fe.npz", E=_np(fe.feature_embedding.weight), x=_np(x), out=_np(out))


def gen_pg(PG):
    res = {}
    g = torch.Generator().manual_seed(8)
    # discount_and_norm_rewards on a sign-reward episode (generate_preds' +-1/0 rewards)
    n = 777
    r = torch.randint(0, 2, (n, 1), generator=g).float()
    r[::7] = -1.0
    r[5] = 0.37
    for gamma in (1.0, 0.9):
        pg = PG.PolicyGradient(100, 6, 1, "g", action_nums=3, reward_decay=gamma, device="cpu")
        pg.ep_rs = r.clone()
        res[f"dn_gamma{gamma}"] = pg.discount_and_norm_rewards()
    res["dn_r"] = _np(r)
    # loss_func and its gradient w.r.t. the policy logits (probs = softmax(logits))
    B, A = 40, 3
    logits = (torch.randn(B, A, generator=g) * 2).requires_grad_(True)
    probs = torch.softmax(logits, dim=1)
    acts = torch.randint(1, A + 1, (B, 1), generator=g)
    vt = torch.randn(B, generator=g)
    loss = pg.loss_func(probs, acts, vt)
    loss.backward()
    res.update(lf_logits=_np(logits), lf_acts=_np(acts), lf_vt=_np(vt),
               lf_loss=np.float32(loss.item()), lf_dlogits=_np(logits.grad))
    # choose_action: net initialised under a known seed, dropout p=0, fixed sampling seed
    torch.manual_seed(11)
    pg = PG.PolicyGradient(100, 6, 1, "g", action_nums=3, device="cpu")
    for mod in pg.policy_net.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    res["ca_param_sums"] = np.array([float(p.detach().double().sum())
                                     for p in pg.policy_net.parameters()])
    res["ca_param_names"] = np.array([k for k, _ in pg.policy_net.named_parameters()])
    x = torch.randint(0, 100, (50, 6), generator=g)
    with torch.no_grad():
        res["ca_probs"] = _np(pg.policy_net(x))
    torch.manual_seed(12)
    res["ca_actions"] = _np(pg.choose_action(x))
    res["ca_x"] = _np(x)
    np.savez(HERE / "g_pg.npz", **res)


def gen_toy_data(d: Path):
    """C1: 1000 rows, 13 dense fields bucketised into 16 ids each + 26 sparse fields of
    50 ids each in one contiguous id space (F=39, V=1508), labels Bernoulli(0.25)."""
    rng = np.random.default_rng(1)
    n, nd, ns, bd, bs = 1000, 13, 26, 16, 50
    dense = rng.lognormal(0.0, 1.0, size=(n, nd))
    edges = np.quantile(dense, np.linspace(0, 1, bd + 1)[1:-1], axis=0)
    cols = []
    for j in range(nd):
        cols.append(j * bd + np.searchsorted(edges[:, j], dense[:, j]))
    zipf = rng.zipf(1.3, size=(n, ns)) - 1
    for j in range(ns):
        cols.append(nd * bd + j * bs + np.minimum(zipf[:, j], bs - 1))
    X = np.stack(cols, axis=1).astype(np.int64)
    y = (rng.random(n) < 0.25).astype(np.int64)
    d.mkdir(parents=True, exist_ok=True)
    rows = np.concatenate([y[:, None], X], axis=1)
    np.savetxt(d / "train_.txt", rows[:800], fmt="%d", delimiter=",")
    np.savetxt(d / "test_.txt", rows[800:], fmt="%d", delimiter=",")
    V = nd * bd + ns * bs
    with open(d / "featindex.txt", "w") as f:
        for i in range(V):
            fld = i // bd if i < nd * bd else nd + (i - nd * bd) // bs
            f.write(f"{fld}:v{i}\t{i}\n")
    return V


_EPOCH_RE = re.compile(r"epoch: (\d+) training average loss: (\S+) validation auc: (\S+) "
                       r"validation loss: (\S+)")


def gen_toy(P, PM, models=("FM", "DeepFM"), merge=False):
    """merge: add `models` to the existing g_toy.json, on the existing toy files."""
    toy = HERE / "toy"
    if merge:
        result = json.loads((HERE / "g_toy.json").read_text())
    else:
        V = gen_toy_data(toy)
        result = {"V": V, "F": 39, "K": 10, "batch_size": 256, "epoch": 5, "lr": 1e-3,
                  "wd": 1e-5}
    for model_name in models:
        with tempfile.TemporaryDirectory() as tmp:
            data_root = Path(tmp) / "data"
            (data_root / "toy").mkdir(parents=True)
            for f in toy.iterdir():
                (data_root / "toy" / f.name).write_bytes(f.read_bytes())
            save_dir = Path(tmp) / "params"
            save_dir.mkdir()
            orig = PM.get_model

            def get_model(*a, **k):  # dropout off so the run is RNG-free and reproducible
                m = orig(*a, **k)
                for mod in m.modules():
                    if isinstance(mod, torch.nn.Dropout):
                        mod.p = 0.0
                return m

            PM.get_model = get_model
            PM.setup_seed(1)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(io.StringIO()):
                PM.main(str(data_root) + "/", "toy/", "", 10, model_name, 5, 1e-3, 1e-5, "loss",
                        256, "cpu", str(save_dir) + "/")
            PM.get_model = orig
            epochs = [dict(epoch=int(m.group(1)), train_loss=float(m.group(2)),
                           valid_auc=float(m.group(3)), valid_loss=float(m.group(4)))
                      for m in _EPOCH_RE.finditer(buf.getvalue())]
            test_auc = float(re.search(r"test auc: (\S+)", buf.getvalue()).group(1))
            sub = data_root / "toy" / model_name / "test_submission.csv"
            preds = [float(line.split(",")[1]) for line in sub.read_text().splitlines()]
            state = torch.load(save_dir / f"{model_name}best.pth", weights_only=True)
            result[model_name] = dict(epochs=epochs, test_auc=test_auc, test_preds=preds,
                                      state_sums={k: float(v.double().sum())
                                                  for k, v in state.items()})
            if model_name == "FM":
                np.savez(HERE / "g_toy_fm_state.npz", **{k: _np(v) for k, v in state.items()})
    (HERE / "g_toy.json").write_text(json.dumps(result, indent=1))


def gen_toy_days(P):
    """toy_days/: the C1 toy rows as ONE train.txt + day_index.csv (days 6..12, ~143 rows
    each; valid day 11, test day 12) for src/main/pretrain_main.py (lr += 1e-4 per epoch);
    g_toy_days.json: its per-epoch log, test AUC and both days' submissions (FM, DeepFM
    with dropout p=0)."""
    import src.main.pretrain_main as PMD  # noqa: E402
    toy, days = HERE / "toy", HERE / "toy_days"
    days.mkdir(exist_ok=True)
    rows = (toy / "train_.txt").read_text() + (toy / "test_.txt").read_text()
    (days / "train.txt").write_text(rows)
    n = len(rows.splitlines())
    bounds = np.linspace(0, n, 8).astype(int)
    with open(days / "day_index.csv", "w") as f:
        for i, d in enumerate(range(6, 13)):
            f.write(f"{d},{bounds[i]},{bounds[i + 1] - 1}\n")
    result = {"valid_day": 11, "test_day": 12, "K": 10, "batch_size": 128, "epoch": 5,
              "lr0": 1e-3, "wd": 1e-5}
    for model_name in ("FM", "DeepFM"):
        with tempfile.TemporaryDirectory() as tmp:
            data_root = Path(tmp) / "data"
            (data_root / "toy_days").mkdir(parents=True)
            for f in days.iterdir():
                (data_root / "toy_days" / f.name).write_bytes(f.read_bytes())
            save_dir = Path(tmp) / "params"
            save_dir.mkdir()
            orig = PMD.get_model

            def get_model(*a, **k):  # dropout off: RNG-free
                m = orig(*a, **k)
                for mod in m.modules():
                    if isinstance(mod, torch.nn.Dropout):
                        mod.p = 0.0
                return m

            PMD.get_model = get_model
            PMD.setup_seed(1)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(io.StringIO()):
                PMD.main(str(data_root) + "/", "toy_days/", "", 11, 12, 10, model_name, 5, 1e-3,
                         1e-5, "loss", 128, "cpu", str(save_dir) + "/")
            PMD.get_model = orig
            epochs = [dict(epoch=int(m.group(1)), train_loss=float(m.group(2)),
                           valid_auc=float(m.group(3)), valid_loss=float(m.group(4)))
                      for m in _EPOCH_RE.finditer(buf.getvalue())]
            test_auc = float(re.search(r"test auc: (\S+)", buf.getvalue()).group(1))
            sub = data_root / "toy_days" / model_name
            preds = {day: [float(line.split(",")[1]) for line in
                           (sub / f"{day}_test_submission.csv").read_text().splitlines()]
                     for day in (11, 12)}
            day_aucs = [[float(x) for x in line.split(",")[1:]]
                        for line in (sub / "day_aucs.csv").read_text().splitlines()]
            result[model_name] = dict(epochs=epochs, test_auc=test_auc, valid_preds=preds[11],
                                      test_preds=preds[12], day_aucs=day_aucs)
    (HERE / "g_toy_days.json").write_text(json.dumps(result, indent=1))


def gen_toy_2(P):
    """g_toy_2.json: src/all_main/pretrain_main_2.py (batches sliced from one preloaded
    LongTensor) on the C1 toy (FM, DeepFM with dropout p=0), 5 epochs."""
    import src.all_main.pretrain_main_2 as PM2  # noqa: E402
    toy = HERE / "toy"
    result = {"K": 10, "batch_size": 256, "epoch": 5, "lr": 1e-3, "wd": 1e-5}
    for model_name in ("FM", "DeepFM"):
        with tempfile.TemporaryDirectory() as tmp:
            data_root = Path(tmp) / "data"
            (data_root / "toy").mkdir(parents=True)
            for f in toy.iterdir():
                (data_root / "toy" / f.name).write_bytes(f.read_bytes())
            save_dir = Path(tmp) / "params"
            save_dir.mkdir()
            orig = PM2.get_model

            def get_model(*a, **k):
                m = orig(*a, **k)
                for mod in m.modules():
                    if isinstance(mod, torch.nn.Dropout):
                        mod.p = 0.0
                return m

            PM2.get_model = get_model
            PM2.setup_seed(1)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(io.StringIO()):
                PM2.main(str(data_root) + "/", "toy/", "", 10, model_name, 5, 1e-3, 1e-5, "loss",
                         256, "cpu", str(save_dir) + "/")
            PM2.get_model = orig
            epochs = [dict(epoch=int(m.group(1)), train_loss=float(m.group(2)),
                           valid_auc=float(m.group(3)), valid_loss=float(m.group(4)))
                      for m in _EPOCH_RE.finditer(buf.getvalue())]
            test_auc = float(re.search(r"test auc: (\S+)", buf.getvalue()).group(1))
            sub = data_root / "toy" / model_name / "test_submission.csv"
            preds = [float(line.split(",")[1]) for line in sub.read_text().splitlines()]
            result[model_name] = dict(epochs=epochs, test_auc=test_auc, test_preds=preds)
    (HERE / "g_toy_2.json").write_text(json.dumps(result, indent=1))


def main():
    P, FE, PG, PM = _import_reference()
    torch.set_num_threads(4)
    gens = {"fm": lambda: gen_fm(P), "deepfm": lambda: gen_deepfm(P), "ipnn": lambda: gen_ipnn(P),
            "ensemble": gen_ensemble, "ffm": lambda: gen_ffm(P),
            "toy_extra": lambda: gen_toy(P, PM, ("IPNN", "FFM"), merge=True),
            "bce": gen_bce, "fe": lambda: gen_fe(FE), "pg": lambda: gen_pg(PG),
            "toy": lambda: gen_toy(P, PM), "toy_days": lambda: gen_toy_days(P),
            "toy_2": lambda: gen_toy_2(P)}
    for name in (sys.argv[1:] or [n for n in gens if n != "toy_extra"] + ["toy_extra"]):
        gens[name]()
    (HERE / "manifest.json").write_text(json.dumps({
        "generator": "tests/golden/make_golden.py",
        "reference": "jqsl2012/RL_CTR_Prediction @ /root/reference (imported, CPU)",
        "torch": torch.__version__, "numpy": np.__version__,
    }, indent=1))
    print("goldens written to", HERE)


if __name__ == "__main__":
    main()
