"""REINFORCE policy of ``src/models/PG_model.py`` on the HIP kernels.

Mirrors ``Net`` (24-58) and ``PolicyGradient`` (60-179): same constructor arguments,
same methods and return types, same CPU RNG calls in ``choose_action`` (so a seeded run
picks the same actions), ``discount_and_norm_rewards`` in fp64 raising
``FloatingPointError`` on a zero std like the reference's ``np.seterr(all='raise')``.

Reference quirk kept by default: ``Net`` sizes its first Linear as
``F(F-1)/2 * K + F*K`` (PG_model.py:34-39) while Feature_Embedding emits
``F(F-1)/2 + F*K`` features, so only latent_dims == 1 runs; any other K raises the
same shape error. ``fix_input_dims=True`` sizes it to the real state width (used for the
C4 REINFORCE configuration; documented in DESIGN.md).

``learn`` is one fused native pass: Feature_Embedding -> 5 fused GEMMs (the three wide
layers on pre-split bf16 planes, csrc/gemm_planes.hip) -> softmax -> loss +
softmax-backward kernel -> 5 weight-gradient GEMMs with Dropout/ReLU mask epilogues ->
dense Adam over one flat parameter buffer; single-process learns replay it as one HIP graph
(Adam scalars and the dropout stream from a device step counter). The embedding is not updated: its
output is detached (Feature_embedding.py:59), so torch's Adam never sees a gradient for it.

Data parallel: the ranks' transitions are slices of ONE episode, in
rank order. Every rank all-gathers the episode's rewards (4 B per transition) and runs the
same discount + normalisation over the whole episode, so the returns, their mean (the
loss_func's mean(vt)) and hence every per-sample logit gradient are bit-identical to one
process learning the whole episode; the weight gradients are summed by one all-reduce
(no division: loss_func is a sum over the episode), the loss shares likewise. Dropout
masks are indexed by the transition's position in the episode, so they match too.
"""
from __future__ import annotations

import os
from contextlib import nullcontext

import numpy as np
import torch
import torch.nn as nn

from . import hip_ops
from .distributed import allgather_varlen, allreduce_sum_, world
from .feature_embedding import Feature_Embedding
from .p_model import _dropout_seed, mlp_forward


class Net(nn.Module):
    def __init__(self, field_nums, feature_nums, latent_dims, action_numbers, campaign_id,
                 fix_input_dims: bool = False):
        super().__init__()
        self.field_nums = field_nums
        self.feature_nums = feature_nums
        self.latent_dims = int(latent_dims)
        self.campaign_id = campaign_id
        self.embedding_layer = Feature_Embedding(self.feature_nums, self.field_nums, self.latent_dims)
        pairs = self.field_nums * (self.field_nums - 1) // 2
        if fix_input_dims:
            input_dims = pairs + self.field_nums * self.latent_dims
        else:  # the reference's formula
            input_dims = pairs * self.latent_dims + self.field_nums * self.latent_dims
        self.input_dims = input_dims
        layers = []
        neuron_nums = 1024
        for _ in range(4):
            layers.append(nn.Linear(input_dims, neuron_nums))
            layers.append(nn.ReLU())
            layers.append(nn.Dropout(p=0.2))
            input_dims = neuron_nums
            neuron_nums = int(neuron_nums / 2)
        layers.append(nn.Linear(input_dims, action_numbers))
        self.mlp = nn.Sequential(*layers)

    def _state(self, x):
        s = self.embedding_layer(x)
        if s.shape[1] != self.input_dims:
            raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({s.shape[0]}x"
                               f"{s.shape[1]} and {self.input_dims}x{self.mlp[0].out_features})")
        return s

    def forward(self, input):
        s = self._state(input)
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.mlp.parameters()):
            return torch.softmax(mlp_forward(self.mlp, s, self.training), dim=1)
        with torch.no_grad():
            logits = mlp_forward(self.mlp, s, self.training)
        return hip_ops.softmax_rows(logits.contiguous())


class _PGLoss(torch.autograd.Function):
    """loss_func's value from the HIP kernel; d loss / d probs for autograd callers."""

    @staticmethod
    def forward(ctx, probs, acts, vt):
        loss, _ = hip_ops.pg_loss_grad(probs.contiguous(), acts, vt)
        ctx.save_for_backward(probs, acts, vt)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        probs, acts, vt = ctx.saved_tensors
        c = vt.reshape(-1).float().mean() * g
        a = acts.reshape(-1, 1).long() - 1
        dp = torch.zeros_like(probs)
        dp.scatter_(1, a, -c / probs.gather(1, a))
        return dp, None, None


class PolicyGradient:
    def __init__(self, feature_nums, field_nums, latent_dims, campaign_id, action_nums=2,
                 learning_rate=1e-4, reward_decay=1, device="cuda:0", fix_input_dims=False,
                 process_group=None):
        self.action_nums = action_nums
        self.feature_nums = feature_nums
        self.field_nums = field_nums
        self.latent_dims = latent_dims
        self.lr = learning_rate
        self.gamma = reward_decay
        self.device = device
        self.campaign_id = campaign_id
        self.group = process_group
        self._ep_states, self._ep_as, self._ep_rs = [], [], []
        self.policy_net = Net(self.field_nums, self.feature_nums, self.latent_dims,
                              self.action_nums, self.campaign_id, fix_input_dims).to(self.device)
        # dense Adam state over one flat buffer holding every MLP parameter
        self._layers = [m for m in self.policy_net.mlp if isinstance(m, nn.Linear)]
        params = [t for lin in self._layers for t in (lin.weight, lin.bias)]
        # 16-B aligned views (offsets multiples of 4 floats) for the GEMMs' float4 path
        n = sum((p.numel() + 3) // 4 * 4 for p in params)
        dev = self._layers[0].weight.device
        self._flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self._grad = torch.zeros_like(self._flat)
        self._m, self._v = torch.zeros_like(self._flat), torch.zeros_like(self._flat)
        self._gviews = []
        self._offsets = []
        off = 0
        for p in params:
            self._offsets.append(off)
            k = p.numel()
            self._flat[off:off + k].copy_(p.data.reshape(-1))
            p.data = self._flat[off:off + k].view_as(p)
            self._gviews.append(self._grad[off:off + k].view_as(p))
            off += (k + 3) // 4 * 4
        self._step = 0
        self.weight_decay = 1e-5  # PG_model.py:87
        self.betas, self.eps = (0.9, 0.999), 1e-8
        self._seed = _dropout_seed()
        # device step counter [completed learns, learn in flight] (advanced by ctr_step_end):
        # the Adam scalars come from the step table and the dropout stream of learn k is
        # (k << 32) + the transition's episode position, so a learn can be captured into a
        # HIP graph and replayed (single process)
        self._step_ctr = torch.tensor([0, 1], dtype=torch.int32, device=dev)
        self._step_done, self._step_cur = self._step_ctr[0:1], self._step_ctr[1:2]
        self._step_table = hip_ops.AdamStepTable(self.lr, self.betas, dev)
        self.use_graphs = True
        self._graphs: dict = {}
        self._graph_pool = torch.cuda.graph_pool_handle()
        # the learn graphs are captured on a stream of this object's own (not torch's shared
        # default capture stream) and every launch takes scratch from its own Workspace: no
        # captured graph shares a scratch buffer with another object's launches
        self._scratch = hip_ops.Workspace()
        self._capture_stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self._graph_tab_version = self._step_table.version
        self._lbufs: dict = {}
        # the layers whose GEMMs run on pre-split bf16 planes (csrc/gemm_planes.hip, the
        # DeepFM MLP's kernel): the wide ones (C4: 741->1024, 1024->512, 512->256 = 97 % of
        # the flops); the narrow tail (256->128->A) stays on ctr_gemm_f32_ex
        self.planes_layers = 0
        if os.environ.get("CTR_PG_PLANES", "1") != "0":
            self.planes_layers = max(0, len(self._layers) - 2)
        self._wplanes = [hip_ops.Planes(l.out_features, l.in_features, dev)
                         for l in self._layers[:self.planes_layers]]
        # weights whose planes the dense Adam rewrites itself (ctr_adam_dense_planes, up to
        # three views, any row length: the 741-wide first layer too); the others are re-split
        # at every learn. _wver: the weights' version counters when their planes were last
        # split (load_state_dict & co. bump them)
        self._adam_planes = list(range(self.planes_layers))[-3:]
        self._wver = None
        self._pbufs: dict = {}
        # the weight-gradient GEMMs (dW_i = g_i^T h_i) on a side stream forked where each g_i
        # is complete, joined before the bias sums and the Adam: the dX chain of the
        # backward keeps the main stream (as the DeepFM step's weight-gradient list)
        # (CTR_PG_WGRAD_SIDE: 0 = off, 1 = every layer, 2 = the planes layers only)
        self._wgrad_side, self._wgrad_mode = None, os.environ.get("CTR_PG_WGRAD_SIDE", "0")
        if self._wgrad_mode != "0" and dev.type == "cuda":
            self._wgrad_side = torch.cuda.Stream(device=dev)

    # ---------------------------------------------------------------- reference API ---
    @property
    def ep_states(self):
        return torch.cat(self._ep_states) if self._ep_states else torch.LongTensor().to(self.device)

    @property
    def ep_as(self):
        return torch.cat(self._ep_as) if self._ep_as else torch.LongTensor().to(self.device)

    @property
    def ep_rs(self):
        return torch.cat(self._ep_rs) if self._ep_rs else torch.FloatTensor().to(self.device)

    @ep_rs.setter
    def ep_rs(self, value):
        self._ep_rs = [value]

    def load_embedding(self, pretrain_params):
        self.policy_net.embedding_layer.feature_embedding.weight.data.copy_(
            torch.from_numpy(np.array(pretrain_params["feature_embedding.weight"].cpu())))

    def loss_func(self, all_act_prob, acts, vt):
        return _PGLoss.apply(all_act_prob, acts.to(all_act_prob.device),
                             vt.to(all_act_prob.device).float())

    def choose_action(self, states):
        prob_weights = self.policy_net.forward(states).cpu()
        random_seeds = torch.rand(len(states), 1)
        max_action = torch.argsort(-prob_weights)[:, 0] + 1
        random_action = torch.randint(low=1, high=self.action_nums + 1, size=[len(states), 1])
        actions = torch.where(random_seeds >= torch.max(prob_weights, 1)[0].view(-1, 1),
                              max_action.view(-1, 1), random_action)
        return actions.to(self.device)

    def choose_best_action(self, state):
        prob_weights = self.policy_net.forward(state)
        return torch.max(prob_weights, 1)[1].view(-1, 1) + 1

    def store_transition(self, s, a, r):
        self._ep_states.append(s)
        self._ep_as.append(a)
        self._ep_rs.append(r)

    def _discount_norm_device(self, out32=None):
        r = self.ep_rs.to(self.device).float().reshape(-1)
        d64, d32, stats = hip_ops.pg_discount_norm(r, float(self.gamma), out32=out32)
        if float(stats[1].item()) == 0.0:
            raise FloatingPointError("divide by zero encountered in divide")
        return d64, d32

    def discount_and_norm_rewards(self):
        d64, _ = self._discount_norm_device()
        return d64.cpu().numpy().reshape(-1, 1)

    def learn(self):
        with self._scratch.scope():  # this object's own scratch (hip_ops.Workspace)
            return self._learn()

    def _learn(self):
        rank, ws = world()
        if ws == 1 and self.use_graphs and self._ep_states and all(
                t.device == self._flat.device for t in self._ep_states + self._ep_as):
            # the inputs are copied into the graph's buffers and the returns written there
            # BEFORE the host waits for the zero-std check (one sync per learn, as the
            # reference raises first), so the GPU idles only for the graph launch after it
            b = self._learn_bufs(None, None)
            self._discount_norm_device(out32=b["vt"])
            loss = self._graph_learn(None, None, None, b=b)
            self._ep_states, self._ep_as, self._ep_rs = [], [], []
            return loss
        states = self.ep_states.to(self.device)
        acts = self.ep_as.to(self.device)
        if ws == 1:
            _, vt = self._discount_norm_device()  # (host check of the zero std: one sync)
            if self.use_graphs and states.is_cuda:
                loss = self._graph_learn(states, acts, vt)
            else:
                self._step_table.ensure(self._step + 1)
                loss = self._fused_learn(states, acts, vt)
                self._step += 1
        else:
            r = self.ep_rs.to(self.device).float().reshape(-1)
            if r.numel() == 0:
                raise ValueError("data-parallel learn: this rank holds no transitions")
            r_all, counts = allgather_varlen(r, self.group)
            _, vt_all, stats = hip_ops.pg_discount_norm(r_all, float(self.gamma))
            if float(stats[1].item()) == 0.0:
                raise FloatingPointError("divide by zero encountered in divide")
            self._step_table.ensure(self._step + 1)
            loss = self._fused_learn(states, acts, None, vt_mean=hip_ops.pg_vt_mean(vt_all),
                                     row0=sum(counts[:rank]), n_episode=sum(counts))
            self._step += 1
        self._ep_states, self._ep_as, self._ep_rs = [], [], []
        return loss

    # ------------------------------------------------------------------ fused pass ----
    def _learn_bufs(self, states, acts) -> dict:
        """The persistent per-episode-size inputs of the learn graph, filled with this
        episode's transitions (states None: straight from the stored ones, one copy)."""
        if states is None:  # straight from the stored transitions (one copy, no cat first)
            n = sum(t.shape[0] for t in self._ep_states)
            F = self._ep_states[0].shape[1]
            sdt = self._ep_states[0].dtype
        else:
            n, F = states.shape
            sdt = states.dtype
        b = self._lbufs.get((n, F))
        if b is None:
            dev = self._flat.device
            b = {"x": torch.empty(n, F, dtype=sdt, device=dev),
                 "a": torch.empty(n, 1, dtype=torch.int64, device=dev),
                 "vt": torch.empty(n, dtype=torch.float32, device=dev)}
            self._lbufs = {(n, F): b}  # the last episode size only
            self._graphs = {k: v for k, v in self._graphs.items() if k[0] == (n, F)}
        if b["x"].dtype != sdt:
            # graphs captured against the old buffer must not replay (their key holds the
            # dtype: switching back would read freed memory)
            torch.cuda.synchronize(self._flat.device)
            self._graphs.clear()
            b["x"] = torch.empty(n, F, dtype=sdt, device=self._flat.device)
        if states is None:
            torch.cat(self._ep_states, out=b["x"])
            torch.cat([a.reshape(-1, 1).to(torch.int64) for a in self._ep_as], out=b["a"])
        else:
            b["x"].copy_(states)
            b["a"].copy_(acts.reshape(n, 1))
        return b

    def _graph_learn(self, states, acts, vt, b=None):
        """_fused_learn on persistent per-episode-size inputs, captured once per (size,
        train mode, dropout) and replayed as a HIP graph (the ~40 launches of a learn).
        b: the inputs already filled by _learn_bufs (vt None: already in b["vt"])."""
        if b is None:
            b = self._learn_bufs(states, acts)
        n, F = b["x"].shape
        if vt is not None:
            b["vt"].copy_(vt.reshape(-1))
        if self._step_table.capacity < self._step + 2:
            self._step_table.ensure(max(self._step + 2, 2 * self._step_table.capacity))
        if self._graph_tab_version != self._step_table.version:
            torch.cuda.synchronize()
            self._graphs.clear()  # they hold the old table's address
            self._graph_tab_version = self._step_table.version
        net = self.policy_net
        drops = tuple(float(net.mlp[3 * i + 2].p) for i in range(4))
        key = ((n, F), b["x"].dtype, net.training, drops, self.planes_layers)
        hit = self._graphs.get(key)
        if hit is None:
            from .trainer import graph_capture, live_pool
            loss = self._fused_learn(b["x"], b["a"], b["vt"])  # the real learn
            self._step += 1
            g = torch.cuda.CUDAGraph()
            with graph_capture(g, pool=live_pool(self), stream=self._capture_stream):
                static = self._fused_learn(b["x"], b["a"], b["vt"])  # captured, not executed
            self._graphs[key] = (g, static)
            return loss
        g, static = hit
        self._sync_planes()
        g.replay()
        self._step += 1
        return static

    def _sync_planes(self) -> None:
        """Re-split the planes layers' weight planes when the fp32 weights changed outside
        the learns (load_state_dict, in-place edits bump the version counters): a replayed
        learn runs the graph captured at the first learn, whose version check ran then."""
        P = self.planes_layers
        if not P:
            return
        ver = tuple(self._layers[i].weight._version for i in range(P))
        if ver != self._wver:
            for i in range(P):
                hip_ops.split_planes(self._layers[i].weight, out=self._wplanes[i])
            self._wver = ver


    def _planes_bufs(self, n: int) -> dict:
        """Per-episode-size buffers of the planes layers: the planes of each layer input
        (hp[i]), the fp32 layer outputs (h[i+1], the dropout / ReLU masks of the backward),
        and the planes of the output gradients (dp[i])."""
        b = self._pbufs.get(n)
        if b is None:
            dev, L, P = self._flat.device, self._layers, self.planes_layers
            e = lambda *sh: torch.empty(*sh, dtype=torch.float32, device=dev)  # noqa: E731
            b = {"hp": [hip_ops.Planes(n, L[i].in_features, dev) for i in range(P)],
                 "h": [None] + [e(n, L[i].out_features) for i in range(P)],
                 "d": [e(n, L[i].out_features) for i in range(P)],
                 "dp": [hip_ops.Planes(n, L[i].out_features, dev) for i in range(P)]}
            self._pbufs = {n: b}  # one episode size at a time (the last one)
        return b

    def _fused_learn(self, states, acts, vt, vt_mean=None, row0: int = 0,
                     n_episode: int | None = None) -> torch.Tensor:
        """vt: this episode's normalised returns (single process); or vt_mean: the
        episode-wide mean(vt) when this rank holds rows [row0, row0 + B) of an episode of
        n_episode transitions split over the data-parallel ranks."""
        net = self.policy_net
        training = net.training
        P = self.planes_layers
        fe = net.embedding_layer
        E = fe.feature_embedding.weight if type(fe) is Feature_Embedding else None
        if (P and E is not None and states.dim() == 2 and
                (lambda F, K: F * (F - 1) // 2 + F * K)(states.shape[1], E.shape[1])
                == net.input_dims):
            # the state and the first planes layer's input planes in one pass (no split)
            pb = self._planes_bufs(states.shape[0])
            x0 = hip_ops.feature_embedding(states, E.detach(), out_planes=pb["hp"][0])
            x0_planes = True
        else:  # (a width mismatch raises the reference's shape error here)
            x0, x0_planes = net._state(states), False
        n = x0.shape[0]
        n_ep = n if n_episode is None else n_episode
        acts_l = []
        h = x0
        mods = list(net.mlp)
        drops = [float(mods[3 * i + 2].p) if training else 0.0 for i in range(4)]
        P = self.planes_layers
        base = 0  # each layer's dropout stream: (learn << 32) + episode position
        if P:
            pb = self._planes_bufs(n)
            ver = tuple(self._layers[i].weight._version for i in range(P))
            for i in range(P):  # the weights' planes from the fp32 parameters: those the
                # Adam keeps current only after an outside change (first learn, load)
                if i not in self._adam_planes or ver != self._wver:
                    hip_ops.split_planes(self._layers[i].weight, out=self._wplanes[i])
            self._wver = ver
            if not x0_planes:
                hip_ops.split_planes(x0.contiguous(), out=pb["hp"][0])
        for i, lin in enumerate(self._layers):
            last = i == len(self._layers) - 1
            off = base + row0 * lin.out_features
            base += n_ep * lin.out_features
            h_in = h
            if i < P:  # same epilogue (bias, ReLU, the same dropout hash) on planes
                p = 0.0 if last else drops[i]
                hip_ops.gemm_planes(pb["hp"][i], self._wplanes[i], False, False,
                                    out=pb["h"][i + 1],
                                    out_planes=pb["hp"][i + 1] if i + 1 < P else None,
                                    epi=hip_ops.EPI_BIAS_RELU_DROP if p > 0 else hip_ops.EPI_BIAS_RELU,
                                    bias=lin.bias, drop_p=p, seed=self._seed, offset=off,
                                    step_dev=self._step_done)
                h = pb["h"][i + 1]
            else:
                h = hip_ops.linear(h_in, lin.weight, lin.bias, relu=not last,
                                   drop_p=0.0 if last else drops[i], seed=self._seed, offset=off,
                                   step_dev=self._step_done)
            acts_l.append(h_in)
        probs = hip_ops.softmax_rows(h)
        if vt_mean is None:
            loss, g = hip_ops.pg_loss_grad(probs, acts, vt)
        else:
            loss, g = hip_ops.pg_loss_grad_global(probs, acts, vt_mean)
        bias_jobs = []
        side = self._wgrad_side if states.is_cuda else None
        held = []  # the side stream's inputs stay referenced until the join
        for i in range(len(self._layers) - 1, -1, -1):
            lin = self._layers[i]
            inp = acts_l[i]
            on_side = side is not None and (self._wgrad_mode != "2" or i < P)
            if on_side:
                side.wait_stream(torch.cuda.current_stream())
                held.append((g, inp))
            with torch.cuda.stream(side) if on_side else nullcontext():
                if i < P:  # g = dL/d(layer i output) is in pb["d"][i] with its planes
                    hip_ops.gemm_planes(pb["dp"][i], pb["hp"][i], True, True,
                                        out=self._gviews[2 * i])
                else:
                    hip_ops.gemm(g, inp, trans_a=True, out=self._gviews[2 * i])
            bias_jobs.append((g, None, self._gviews[2 * i + 1]))  # db = colsum g
            if i > 0:
                sc = 1.0 / (1.0 - drops[i - 1])
                if i - 1 < P:  # the next layer down runs on planes: write g's planes too
                    if i < P:
                        hip_ops.gemm_planes(pb["dp"][i], self._wplanes[i], False, True,
                                            out=pb["d"][i - 1], out_planes=pb["dp"][i - 1],
                                            epi=hip_ops.EPI_GRAD_MASK, aux=inp, scale=sc)
                    else:
                        hip_ops.gemm(g, lin.weight, epi=hip_ops.EPI_GRAD_MASK, aux=inp, scale=sc,
                                     out=pb["d"][i - 1])
                        hip_ops.split_planes(pb["d"][i - 1], out=pb["dp"][i - 1])
                    g = pb["d"][i - 1]
                else:
                    g = hip_ops.gemm(g, lin.weight, epi=hip_ops.EPI_GRAD_MASK, aux=inp,
                                     scale=sc)
        if side is not None:
            torch.cuda.current_stream().wait_stream(side)
        del held
        hip_ops.colsum_multi(bias_jobs)  # the five bias gradients in one launch pair
        if vt_mean is not None:  # the episode's gradient and loss: sums of the ranks' shares
            allreduce_sum_(self._grad, self.group)
            allreduce_sum_(loss, self.group)
        planes = [(self._offsets[2 * i], self._wplanes[i]) for i in self._adam_planes]
        hip_ops.adam_dense(self._flat, self._grad, self._m, self._v, self._step + 1, self.lr,
                           self.betas, self.eps, self.weight_decay, step_dev=self._step_cur,
                           table=self._step_table, planes=planes or None)
        hip_ops.step_end(self._step_ctr)
        return loss
