"""CPU oracle for the CTR hot path — TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may import this
module, and only as the checker / the timed CPU baseline. The product path
(rl_ctr_prediction_amd) never imports it and has no CPU fallback.

A from-scratch restatement of jqsl2012/RL_CTR_Prediction's algorithms on torch-CPU
(the reference's own runtime) + numpy, written functionally from SURVEY.md §8a:

  fm_forward          p_model.py:40-57       (FM.forward)
  deepfm_forward      p_model.py:296-324     (DeepFM.to_fm + forward, MLP 276-293)
  ipnn_forward        p_model.py:146-200     (InnerPNN: flat ++ pairwise inner products, MLP)
  ffm_forward         p_model.py:59-100      (FFM: one table per field, E_j[x_i] . E_i[x_j])
  bce                 all_main/pretrain_main.py:74,139 (nn.BCELoss, mean)
  train_step          all_main/pretrain_main.py:67-83 (fwd, BCE, zero_grad, backward, Adam)
  feature_embedding   Feature_embedding.py:51-59
  pg_*                PG_model.py:104-154 (loss_func, choose_action, discount_and_norm)
  pg_policy/pg_learn  PG_model.py:24-58,156-179 (Net, learn: FE state, MLP, loss, Adam)
  ensemble_preds      all_main/hybrid_td3_main_per_v10.py:54-164 (generate_preds, per example)
  sparse_plan         the grouping inside embedding_dense_backward (numpy, bit-exact ints)
  pretrain_run        all_main/pretrain_main.py:119-202 (per-epoch Adam, no shuffle, AUC)

Parity is PINNED: tests/test_oracle.py checks every function here against the golden
vectors in tests/golden/, produced by importing the reference itself
(tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as Fn

# ---------------------------------------------------------------- parameters --------
FM_KEYS = ("bias", "linear.weight", "feature_embedding.weight")
DEEPFM_KEYS = FM_KEYS + ("mlp.0.weight", "mlp.0.bias", "mlp.3.weight", "mlp.3.bias",
                         "mlp.6.weight", "mlp.6.bias")


IPNN_KEYS = ("feature_embedding.weight", "mlp.0.weight", "mlp.0.bias", "mlp.3.weight",
             "mlp.3.bias", "mlp.6.weight", "mlp.6.bias")


def ipnn_pairs(F: int):
    """The reference's self.row / self.col (p_model.py:179-182): row-major i < j."""
    row, col = np.triu_indices(F, k=1)
    return torch.as_tensor(row), torch.as_tensor(col)


def init_params(kind: str, V: int, F: int, K: int, seed: int | None = None) -> dict:
    """Parameters with the reference modules' default initialisers, created in the
    reference's order: N(0,1) embeddings (nn.Embedding), zero bias, nn.Linear's
    kaiming-uniform weights / uniform biases."""
    if seed is not None:
        torch.manual_seed(seed)
    if kind == "FFM":  # p_model.py:65-78: linear, bias, then one Embedding(V, K) per field
        p = {"linear.weight": torch.nn.Embedding(V, 1).weight.data, "bias": torch.zeros(1)}
        for t in range(F):
            p[f"field_feature_embeddings.{t}.weight"] = torch.nn.Embedding(V, K).weight.data
        return {k: v.clone().requires_grad_(True) for k, v in p.items()}
    if kind == "IPNN":  # p_model.py:153-177: embedding, then Linear(F*K + P, 300), ...
        p = {"feature_embedding.weight": torch.nn.Embedding(V, K).weight.data}
        dims = [F * K + F * (F - 1) // 2, 300, 200, 1]
        for i, name in zip(range(3), ("mlp.0", "mlp.3", "mlp.6")):
            lin = torch.nn.Linear(dims[i], dims[i + 1])
            p[f"{name}.weight"] = lin.weight.data
            p[f"{name}.bias"] = lin.bias.data
        return {k: v.clone().requires_grad_(True) for k, v in p.items()}
    p = {"linear.weight": torch.nn.Embedding(V, 1).weight.data,
         "bias": torch.zeros(1),
         "feature_embedding.weight": torch.nn.Embedding(V, K).weight.data}
    if kind == "DeepFM":
        dims = [F * K, 300, 200, 1]
        for i, name in zip(range(3), ("mlp.0", "mlp.3", "mlp.6")):
            lin = torch.nn.Linear(dims[i], dims[i + 1])
            p[f"{name}.weight"] = lin.weight.data
            p[f"{name}.bias"] = lin.bias.data
    return {k: v.clone().requires_grad_(True) for k, v in p.items()}


# ------------------------------------------------------------------ forward ---------
def fm_logit(params: dict, x: torch.Tensor) -> torch.Tensor:
    """bias + sum_f w[x_f] + 0.5 * sum_k((sum_f e_fk)^2 - sum_f e_fk^2), shape [B,1]."""
    e = Fn.embedding(x, params["feature_embedding.weight"])            # [B,F,K]
    square_of_sum = e.sum(dim=1) ** 2
    sum_of_square = (e ** 2).sum(dim=1)
    inter = (square_of_sum - sum_of_square).sum(dim=1, keepdim=True)
    lin = Fn.embedding(x, params["linear.weight"]).sum(dim=1)            # [B,1]
    return params["bias"] + lin + inter * 0.5


def fm_forward(params: dict, x: torch.Tensor) -> torch.Tensor:
    return torch.sigmoid(fm_logit(params, x))


def mlp(params: dict, h: torch.Tensor, drop_p: float, training: bool) -> torch.Tensor:
    for name in ("mlp.0", "mlp.3"):
        h = Fn.relu(Fn.linear(h, params[f"{name}.weight"], params[f"{name}.bias"]))
        h = Fn.dropout(h, p=drop_p, training=training)
    return Fn.linear(h, params["mlp.6.weight"], params["mlp.6.bias"])


def deepfm_forward(params: dict, x: torch.Tensor, drop_p: float = 0.2,
                   training: bool = True) -> torch.Tensor:
    B, F = x.shape
    e = Fn.embedding(x, params["feature_embedding.weight"])
    deep = mlp(params, e.reshape(B, -1), drop_p, training)
    return torch.sigmoid(fm_logit(params, x) + deep)


def ipnn_cat(E: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """MLP input of InnerPNN.forward (p_model.py:187-195): flat(e) ++ <e_i, e_j>, i < j."""
    B, F = x.shape
    e = Fn.embedding(x, E)
    row, col = ipnn_pairs(F)
    inner = torch.sum(torch.mul(e[:, row], e[:, col]), dim=2)
    return torch.cat([e.reshape(B, -1), inner], dim=1)


def ipnn_forward(params: dict, x: torch.Tensor, drop_p: float = 0.2,
                 training: bool = True) -> torch.Tensor:
    return torch.sigmoid(mlp(params, ipnn_cat(params["feature_embedding.weight"], x), drop_p,
                             training))


def ffm_logit(params: dict, x: torch.Tensor) -> torch.Tensor:
    """bias + sum_f w[x_f] + sum_k sum_{i<j} E_j[x_i,k] * E_i[x_j,k], shape [B,1]."""
    B, F = x.shape
    emb = [Fn.embedding(x, params[f"field_feature_embeddings.{t}.weight"]) for t in range(F)]
    row, col = ipnn_pairs(F)
    second = torch.stack([emb[j][:, i] * emb[i][:, j]
                          for i, j in zip(row.tolist(), col.tolist())], dim=1)  # [B, P, K]
    lin = Fn.embedding(x, params["linear.weight"]).sum(dim=1)
    return params["bias"] + lin + second.sum(dim=1).sum(dim=1, keepdim=True)


def forward(kind: str, params: dict, x, drop_p=0.2, training=True):
    if kind == "FFM":
        return torch.sigmoid(ffm_logit(params, x))
    if kind == "FM":
        return fm_forward(params, x)
    if kind == "IPNN":
        return ipnn_forward(params, x, drop_p, training)
    return deepfm_forward(params, x, drop_p, training)


def bce(p: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    return Fn.binary_cross_entropy(p, y)


# ---------------------------------------------------------------- training ---------
def make_optimizer(params: dict, lr: float, weight_decay: float):
    """torch.optim.Adam over the parameters (reference: all_main/pretrain_main.py:153),
    in state_dict order so the optimiser state lines up with the reference's."""
    return torch.optim.Adam(list(params.values()), lr=lr, weight_decay=weight_decay)


def train_step(kind: str, params: dict, opt, x: torch.Tensor, y: torch.Tensor,
               drop_p: float = 0.2, split: dict | None = None) -> float:
    """One reference step: forward, BCE, zero_grad, backward (dense embedding grads),
    Adam.step, loss.item()  (all_main/pretrain_main.py:72-79). split: accumulates the
    seconds of the forward (+ BCE), backward and optimizer phases (BASELINE.md protocol)."""
    import time
    t0 = time.perf_counter()
    p = forward(kind, params, x, drop_p, True)
    loss = bce(p, y.reshape(-1, 1).to(p.dtype))
    t1 = time.perf_counter()
    for t in params.values():
        t.grad = None
    loss.backward()
    t2 = time.perf_counter()
    opt.step()
    t3 = time.perf_counter()
    if split is not None:
        for k, d in (("fwd", t1 - t0), ("bwd", t2 - t1), ("adam", t3 - t2)):
            split[k] = split.get(k, 0.0) + d
    return loss.item()


def grads(kind: str, params: dict, x, y, drop_p=0.0) -> tuple[float, torch.Tensor, dict]:
    p = forward(kind, params, x, drop_p, True)
    loss = bce(p, y.reshape(-1, 1).to(p.dtype))
    for t in params.values():
        t.grad = None
    loss.backward()
    return loss.item(), p.detach(), {k: v.grad.clone() for k, v in params.items()}


def grad_condition(kind: str, params: dict, x: torch.Tensor, y: torch.Tensor) -> dict:
    """First-order L1 condition of each embedding-gradient element: the sum of |summand|
    over every rounded operation that feeds it, so |fp32 error| <= ~u * A regardless of
    cancellation (used as the parity scale of a gradient, tests/conftest.py).

    The reference's gradient of slot (b,f) is g_b*s_bk - g_b*e_bfk (FM; g = dL/dz,
    s = sum_f e: a K-column sum whose own rounding depends on summation order, so its
    condition is sum_f |e_bfk|, not |s_bk|) plus the MLP-input gradient dX = dH1 @ W0 with
    dH1 = mask * (dH2 @ W1) (condition |dH2| @ |W1| @ |W0| through the ReLU mask); a row
    sums these over up to ~1e4 slots, so
    A[r,k] = sum over the row's slots of |g_b|*sum_f|e_bfk| + |g_b*e_bfk| + mlp_cond_bfk.
    Dropout off."""
    B, F = x.shape
    E = params["feature_embedding.weight"].detach()
    V, K = E.shape
    if kind == "IPNN":
        return _ipnn_condition(params, x, y)
    w = params["linear.weight"].detach()
    e = Fn.embedding(x, E)
    lw = Fn.embedding(x, w).detach()
    s = e.sum(dim=1)
    inter = ((s ** 2) - (e ** 2).sum(dim=1)).sum(dim=1, keepdim=True)
    z = (params["bias"].detach() + lw.sum(dim=1) + inter * 0.5).requires_grad_(True)
    zt = z
    if kind == "DeepFM":
        det = {k: v.detach() for k, v in params.items()}
        h1 = Fn.relu(Fn.linear(e.reshape(B, -1), det["mlp.0.weight"], det["mlp.0.bias"]))
        h2 = Fn.relu(Fn.linear(h1, det["mlp.3.weight"], det["mlp.3.bias"]))
        zt = z + Fn.linear(h2, det["mlp.6.weight"], det["mlp.6.bias"])
    bce(torch.sigmoid(zt), y.reshape(-1, 1).float()).backward()
    g = z.grad.reshape(B, 1, 1)                                   # dL/dz per example
    terms = g.abs() * e.abs().sum(dim=1, keepdim=True) + (g * e).abs()   # [B,F,K]
    if kind == "DeepFM":
        dh2 = (g.reshape(B, 1) * det["mlp.6.weight"]).abs() * (h2 > 0)      # [B,200]
        c1 = (dh2 @ det["mlp.3.weight"].abs()) * (h1 > 0)                  # [B,300]
        terms = terms + (c1 @ det["mlp.0.weight"].abs()).reshape(B, F, K)
    flat = x.reshape(-1)
    A_E = torch.zeros(V, K).index_add_(0, flat, terms.reshape(-1, K))
    A_w = torch.zeros(V, 1).index_add_(0, flat, g.reshape(B, 1).abs().expand(B, F).reshape(-1, 1))
    return {"feature_embedding.weight": A_E, "linear.weight": A_w}


def _ipnn_condition(params: dict, x: torch.Tensor, y: torch.Tensor) -> dict:
    """grad_condition for InnerPNN: dz = dL/dz per example; the condition of dcat is
    |dz| |W2| |W1| |W0| through the ReLU masks; a slot's gradient sums its flat part and
    sum_j dP_fj e_j, whose condition is (cond(dP_fj) + |dP_fj|) |e_j|."""
    B, F = x.shape
    det = {k: v.detach() for k, v in params.items()}
    E = det["feature_embedding.weight"]
    V, K = E.shape
    cat = ipnn_cat(E, x)
    h1 = Fn.relu(Fn.linear(cat, det["mlp.0.weight"], det["mlp.0.bias"]))
    h2 = Fn.relu(Fn.linear(h1, det["mlp.3.weight"], det["mlp.3.bias"]))
    z = Fn.linear(h2, det["mlp.6.weight"], det["mlp.6.bias"]).requires_grad_(True)
    bce(torch.sigmoid(z), y.reshape(-1, 1).float()).backward()
    g = z.grad.reshape(B, 1)
    dh2 = (g * det["mlp.6.weight"]).abs() * (h2 > 0)
    c1 = (dh2 @ det["mlp.3.weight"].abs()) * (h1 > 0)
    ccat = c1 @ det["mlp.0.weight"].abs()                                  # [B, F*K + P]
    d1 = (g * det["mlp.6.weight"]) * (h2 > 0)
    dcat = (((d1 @ det["mlp.3.weight"]) * (h1 > 0)) @ det["mlp.0.weight"]).abs()
    e = Fn.embedding(x, E).abs()                                           # [B, F, K]
    terms = ccat[:, :F * K].reshape(B, F, K).clone()
    row, col = ipnn_pairs(F)
    wp = ccat[:, F * K:] + dcat[:, F * K:]                                 # [B, P]
    for p_, (i, j) in enumerate(zip(row.tolist(), col.tolist())):
        terms[:, i] += wp[:, p_:p_ + 1] * e[:, j]
        terms[:, j] += wp[:, p_:p_ + 1] * e[:, i]
    A_E = torch.zeros(V, K).index_add_(0, x.reshape(-1), terms.reshape(-1, K))
    return {"feature_embedding.weight": A_E}


# ------------------------------------------------------- RL ensemble (generate_preds) --
def ensemble_preds(preds, actions, prob_weights, c_actions, labels):
    """generate_preds (hybrid_td3_main_per_v10.py:54-164) restated per example, fp32 like the
    reference's tensors: preds/prob_weights/c_actions [B,M], actions [B] (1-based ensemble
    size), labels [B]. Returns (y [B], rewards [B], return_c_actions [B,M]) as float32.

    a == M: y = sum_m pw*pred, ret_c = c. a < M: the a models with the largest pw (stable
    order), softmax of the a largest c values of the example, y = sum w*pred; ret_c[model_m]
    = m-th largest c value of batch row j, j = the example's ordinal among same-action
    examples (the reference indexes the full-batch sorted c_actions with group-local
    positions, line 127). Reward: label 1 -> y > mean(preds), label 0 -> y < mean."""
    preds = np.asarray(preds, np.float32)
    pw = np.asarray(prob_weights, np.float32)
    ca = np.asarray(c_actions, np.float32)
    act = np.asarray(actions).reshape(-1)
    lab = np.asarray(labels).reshape(-1)
    B, M = preds.shape
    y = np.ones(B, np.float32)
    r = np.ones(B, np.float32)
    rc = np.zeros((B, M), np.float32)
    seen = {}
    for b in range(B):
        a = int(act[b])
        if not 1 <= a <= M:
            continue
        j = seen.get(a, 0)
        seen[a] = j + 1
        mean = np.float32(preds[b].sum(dtype=np.float32) / np.float32(M))
        if a == M:
            acc = np.float32(0)
            for m in range(M):
                acc = np.float32(acc + np.float32(pw[b, m] * preds[b, m]))
            y[b] = acc
            rc[b] = ca[b]
        else:
            models = np.argsort(-pw[b], kind="stable")[:a]
            top_c = np.sort(ca[b])[::-1][:a]
            row_j = np.sort(ca[j])[::-1]
            e = np.exp((top_c - top_c[0]).astype(np.float64)).astype(np.float32)
            w = (e / e.sum(dtype=np.float32)).astype(np.float32)
            acc = np.float32(0)
            for m in range(a):
                acc = np.float32(acc + np.float32(w[m] * preds[b, models[m]]))
                rc[b, models[m]] = row_j[m]
            y[b] = acc
        if lab[b] == 1:
            r[b] = 1.0 if y[b] > mean else 0.0
        elif lab[b] == 0:
            r[b] = 1.0 if y[b] < mean else 0.0
    return y, r, rc


# ------------------------------------------------------------ scatter grouping -------
def sparse_plan(x: np.ndarray):
    """Stable grouping of slots by id: (sorted_slots, sorted_rows, pos_seg, unique_rows,
    seg_offsets) — what ctr_sparse_plan_build must reproduce bit-exactly."""
    flat = np.asarray(x).reshape(-1).astype(np.int64)
    order = np.argsort(flat, kind="stable")
    rows = flat[order]
    uniq, first, counts = np.unique(rows, return_index=True, return_counts=True)
    offsets = np.concatenate([first, [flat.size]]).astype(np.int64)
    pos_seg = np.repeat(np.arange(uniq.size), counts)
    return order, rows, pos_seg, uniq, offsets


# -------------------------------------------------------------- Feature_Embedding ----
def feature_embedding(E: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    B, F = x.shape
    e = Fn.embedding(x, E)
    i, j = np.triu_indices(F, k=1)          # row-major pairs (i<j), Feature_embedding.py:40-43
    inner = (e[:, i] * e[:, j]).sum(dim=2)
    return torch.cat([inner, e.reshape(B, -1)], dim=1).detach()


# -------------------------------------------------------------------- REINFORCE -----
def pg_discount_and_norm(r: np.ndarray, gamma: float) -> np.ndarray:
    """Reverse discounted return in float64, then (d - mean) / std (PG_model.py:139-154)."""
    r = np.asarray(r, dtype=np.float32).reshape(-1)
    d = np.zeros(r.shape + (1,), dtype=np.float64)
    run = 0.0
    for i in range(r.size - 1, -1, -1):
        run = run * gamma + float(r[i])
        d[i] = run
    d -= np.mean(d)
    std = np.std(d)
    if std == 0:
        raise FloatingPointError("divide by zero encountered in divide")
    d /= std
    return d


def pg_loss(probs: torch.Tensor, acts: torch.Tensor, vt: torch.Tensor) -> torch.Tensor:
    """sum_b(-log p[b, a_b-1]) * mean(vt)  (PG_model.py:104-107; acts are 1-based)."""
    nlp = torch.sum(-torch.log(probs.gather(1, acts.reshape(-1, 1).long() - 1)))
    return torch.mean(nlp * vt)


def pg_choose_action(probs: torch.Tensor, action_nums: int) -> torch.Tensor:
    """PG_model.py:110-121 on host probabilities (same CPU RNG calls, same order)."""
    n = probs.shape[0]
    random_seeds = torch.rand(n, 1)
    max_action = torch.argsort(-probs)[:, 0] + 1
    random_action = torch.randint(low=1, high=action_nums + 1, size=[n, 1])
    return torch.where(random_seeds >= torch.max(probs, 1)[0].view(-1, 1),
                       max_action.view(-1, 1), random_action)


def pg_policy(input_dims: int, action_nums: int) -> torch.nn.Sequential:
    """Net.mlp (PG_model.py:41-56): [Linear -> ReLU -> Dropout(0.2)] x 4 with widths
    1024, 512, 256, 128, then Linear(action_nums); softmax applied by the caller."""
    layers, width, d = [], 1024, input_dims
    for _ in range(4):
        layers += [torch.nn.Linear(d, width), torch.nn.ReLU(), torch.nn.Dropout(p=0.2)]
        d, width = width, width // 2
    layers.append(torch.nn.Linear(d, action_nums))
    return torch.nn.Sequential(*layers)


def pg_learn(policy: torch.nn.Sequential, opt, E: torch.Tensor, states: torch.Tensor,
             acts: torch.Tensor, rewards: np.ndarray, gamma: float = 1.0) -> float:
    """PolicyGradient.learn (PG_model.py:156-179): returns, FE state (detached), softmax
    policy, loss_func, zero_grad/backward/Adam.step (Adam(lr 1e-4, wd 1e-5), line 87)."""
    vt = torch.from_numpy(pg_discount_and_norm(rewards, gamma)).float()
    probs = torch.softmax(policy(feature_embedding(E, states)), dim=1)
    loss = pg_loss(probs, acts, vt)
    opt.zero_grad()
    loss.backward()
    opt.step()
    return loss.item()


# --------------------------------------------------------------------- driver -------
def pretrain_run(kind: str, train: np.ndarray, test: np.ndarray, V: int, K: int, epochs: int,
                 lr: float, wd: float, batch: int, seed: int = 1, drop_p: float = 0.0,
                 lr_step: float = 0.0, dtype=torch.float32, extra_eval=()):
    """all_main/pretrain_main.main without files: Adam re-created every epoch, batches in
    file order, train loss = mean of batch losses, AUC over the test split.
    lr_step: main/pretrain_main.py:180 adds 1e-4 to the learning rate before every epoch.
    dtype=torch.float64 replays the same run (same fp32 initial values) in double precision:
    the exact-arithmetic trajectory the fp32 reference's rounding is measured against.
    The last epoch's dict carries the eval split's predictions ("preds") and those of every
    extra_eval matrix ("extra_preds"; the driver's test_submission of a run without early stop)."""
    from sklearn.metrics import roc_auc_score
    F = train.shape[1] - 1
    params = init_params(kind, V, F, K, seed=seed)
    if dtype != torch.float32:
        params = {k: v.detach().to(dtype).requires_grad_(True) for k, v in params.items()}
    hist = []
    xt = torch.from_numpy(test[:, 1:]).long()
    yt = torch.from_numpy(test[:, 0]).to(dtype)
    for _ in range(epochs):
        lr += lr_step
        opt = make_optimizer(params, lr, wd)
        losses = []
        for s in range(0, len(train), batch):
            xb = torch.from_numpy(train[s:s + batch, 1:]).long()
            yb = torch.from_numpy(train[s:s + batch, 0]).to(dtype)
            losses.append(train_step(kind, params, opt, xb, yb, drop_p))
        with torch.no_grad():
            preds, vl = [], []
            for s in range(0, len(test), batch):
                p = forward(kind, params, xt[s:s + batch], drop_p, False)
                vl.append(bce(p, yt[s:s + batch].reshape(-1, 1)).item())
                preds.append(p.reshape(-1))
            pr = torch.cat(preds).numpy()
        hist.append(dict(train_loss=sum(losses) / len(losses),
                         valid_auc=float(roc_auc_score(test[:, 0], pr)),
                         valid_loss=sum(vl) / len(vl)))
    with torch.no_grad():
        hist[-1]["preds"] = pr
        hist[-1]["extra_preds"] = [
            torch.cat([forward(kind, params, torch.from_numpy(m[s:s + batch, 1:]).long(), drop_p,
                               False).reshape(-1) for s in range(0, len(m), batch)]).numpy()
            for m in extra_eval]
    return hist, params
