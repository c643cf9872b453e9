"""The fused FFM training step: the reference's per-batch body
(all_main/pretrain_main.py:72-79: ``y = model(x); loss = BCELoss(y, labels);
model.zero_grad(); loss.backward(); optimizer.step()``) for FFM (p_model.py:59-100) with
torch.optim.Adam(lr, weight_decay) — dense Adam semantics (every row of every field table
moves every step), computed deferred-exact like FusedCTRTrainer's default mode.

The F field tables ``field_feature_embeddings.t.weight`` [V, K] are re-pointed into one
contiguous [F*V, K] buffer (same Parameter objects, same state_dict), so the F*V
(table, row) key space of ctr_ffm_backward is one deferred-Adam table:

  ffm_keys(x)                      keys t*V + x[b,f] of every (example, field, table) slot
  sparse plans over keys and x     (the field tables' and the linear table's rows)
  deferred catch-up of those rows  (they replay the g = wd*p steps they missed)
  ffm_forward(+BCE head)           z, p, per-example loss, dL/dz
  ffm_backward                     per-slot table-row gradients [B*F*(F-1), K]
  segmented sums (+ Adam apply)    per (table, row), in slot order, applied at step t
  linear: per-row sums of dL/dz    + its deferred Adam; bias: sum(dL/dz) + dense Adam

No dense [F*V, K] gradient is materialised (the AutogradTrainer path writes F dense [V, K]
gradients and streams F*V*K*24 B of Adam traffic per step). Single-process steps are
captured into HIP graphs and replayed, as in FusedCTRTrainer.step.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.nn as nn

from . import hip_ops
from .p_model import FFM
from .trainer import flush_hooks, graph_capture, live_pool


@dataclass
class _FFMBufs:
    B: int
    keys: torch.Tensor                 # int32 [S2]  S2 = B*F*(F-1)
    vals: torch.Tensor                 # [S2, K]     per-slot table-row gradients
    plan: hip_ops.SparsePlanBuffers    # over keys (F*V rows)
    plan_x: hip_ops.SparsePlanBuffers  # over x (V rows of the linear table)
    grad_rows: torch.Tensor            # [S2, K]     per-row sums (scratch)
    slot_g: torch.Tensor               # [B*F, 1]    dL/dz of each slot's example
    grad_w: torch.Tensor               # [B*F, 1]    per-row sums of the linear table
    fwd: dict                          # z, p, loss_elem, gz [B]
    loss: torch.Tensor                 # [1]


class FusedFFMTrainer:
    """Fused forward + BCE + backward + deferred-exact dense Adam for FFM.

    Args mirror ``torch.optim.Adam(model.parameters(), lr, betas, eps, weight_decay)``;
    the interface is FusedCTRTrainer's (step / flush / reset_optimizer /
    optimizer_state_dict / check_errors)."""

    def __init__(self, model: nn.Module, lr: float = 1e-3, weight_decay: float = 0.0,
                 betas=(0.9, 0.999), eps: float = 1e-8, seed: int | None = None):
        if not isinstance(model, FFM):
            raise TypeError("FusedFFMTrainer drives FFM")
        tabs = [e.weight for e in model.field_feature_embeddings]
        self.model = model
        self.kind = "FFM"
        self.lr, self.weight_decay, self.betas, self.eps = float(lr), float(weight_decay), betas, eps
        self.device = tabs[0].device
        if self.device.type != "cuda":
            raise RuntimeError("FusedFFMTrainer needs the model on a ROCm device")
        self.F = len(tabs)
        self.V, self.K = tabs[0].shape
        if self.F < 2:
            raise ValueError("FusedFFMTrainer: FFM needs at least 2 fields")
        if self.F * self.V >= 2**31:
            raise ValueError("FusedFFMTrainer: F*V must fit int32 keys")
        FV, K, dev = self.F * self.V, self.K, self.device
        # the field tables as row blocks of one [F*V, K] table
        self.T = torch.empty(FV, K, dtype=torch.float32, device=dev)
        for t, p in enumerate(tabs):
            blk = self.T[t * self.V:(t + 1) * self.V]
            blk.copy_(p.data)
            p.data = blk
        self.m_T = torch.zeros_like(self.T)
        self.v_T = torch.zeros_like(self.T)
        self.last_T = torch.zeros(FV, dtype=torch.int32, device=dev)
        # the linear table [V, 1] as a K = 1 deferred table; the bias through the dense Adam
        self.w = model.linear.weight.data
        self.m_w = torch.zeros_like(self.w)
        self.v_w = torch.zeros_like(self.w)
        self.last_w = torch.zeros(self.V, dtype=torch.int32, device=dev)
        self.bias = model.bias.data
        self.g_bias = torch.zeros_like(self.bias)
        self.m_b = torch.zeros_like(self.bias)
        self.v_b = torch.zeros_like(self.bias)
        self.ptrs = model._ptrs.get(tabs)
        self._vec_ok = K % 4 == 0 and 64 % (K // 4 or 1) == 0 and K <= 256
        self.fuse_apply = os.environ.get("CTR_FUSE_APPLY", "1") != "0"
        self.keep_grads = False  # fused apply: keep every row's sum in b.grad_rows (tests)
        self.step_ctr = torch.tensor([0, 1], dtype=torch.int32, device=dev)
        self.step_done, self.step_cur = self.step_ctr[0:1], self.step_ctr[1:2]
        self.step_table = hip_ops.AdamStepTable(self.lr, self.betas, dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.loss_sum = torch.zeros(1, dtype=torch.float64, device=dev)
        # own scratch and capture stream (hip_ops.Workspace: no captured graph shares
        # scratch with another object's launches)
        self._scratch = hip_ops.Workspace()
        self._capture_stream = torch.cuda.Stream(device=dev)
        self.step_count = 0
        self._dirty = False
        flush_hooks(model, self)
        self._bufs: _FFMBufs | None = None
        self._bufsets: dict = {}
        self.seed = int(torch.initial_seed() if seed is None else seed) & (2**63 - 1)
        self.use_graphs = True
        self.max_graphs = 8
        self._graphs: dict = {}
        # every batch is copied into the fixed input buffers of its shape (ids, labels), so
        # one captured graph per shape serves a stream of fresh batches
        self._inputs: dict = {}
        self.captures = 0
        # bounded staleness, as FusedCTRTrainer.flush_every
        self.flush_every = int(os.environ.get("CTR_FLUSH_EVERY", "32"))
        self._flushed_at = 0
        self._graph_pool = torch.cuda.graph_pool_handle()
        self._graph_tab_version = self.step_table.version
        self.timing = None  # FusedCTRTrainer's bench hook: not instrumented here

    def __del__(self):
        try:  # a captured graph must not be destroyed while it still runs
            if getattr(self, "_graphs", None):
                torch.cuda.synchronize(self.device)
        except Exception:  # interpreter shutdown
            pass

    # ----------------------------------------------------------------- optimiser -----
    def _table_args(self):
        return (self.T, self.m_T, self.v_T, None, None, None, self.last_T)

    def _w_args(self):
        return (self.w, self.m_w, self.v_w, None, None, None, self.last_w)

    def flush(self) -> None:
        """Bring every row of every table up to the last completed step."""
        self._flushed_at = self.step_count
        if self._dirty and self.step_count > 0:
            for tab in (self._table_args(), self._w_args()):
                hip_ops.adam_deferred_flush(*tab, self.step_count, self.step_table, self.betas,
                                            self.eps, self.weight_decay)
        self._dirty = False

    def reset_optimizer(self, lr: float | None = None) -> None:
        """A re-created torch.optim.Adam (all_main/pretrain_main.py:153), optionally at a new
        learning rate; captured graphs stay valid (the step table is rewritten in place)."""
        self.flush()
        if lr is not None:
            self.lr = float(lr)
            self.step_table.set_lr(self.lr)
        for t in (self.m_T, self.v_T, self.m_w, self.v_w, self.m_b, self.v_b, self.last_T,
                  self.last_w):
            t.zero_()
        self.step_ctr.copy_(torch.tensor([0, 1], dtype=torch.int32))
        self.step_count = 0
        self._flushed_at = 0

    def optimizer_state_dict(self) -> dict:
        """torch.optim.Adam-compatible state_dict: parameter i is the i-th entry of
        model.named_parameters() (for FFM: bias first — a root module's own parameters come
        before its submodules' —, then linear.weight and the field tables)."""
        self.flush()
        V = self.V
        moments = {"bias": (self.m_b, self.v_b), "linear.weight": (self.m_w, self.v_w)}
        for t in range(self.F):
            sl = slice(t * V, (t + 1) * V)
            moments[f"field_feature_embeddings.{t}.weight"] = (self.m_T[sl], self.v_T[sl])
        named = [n for n, _ in self.model.named_parameters()]
        state = {i: {"step": torch.tensor(float(self.step_count)),
                     "exp_avg": moments[n][0].clone(), "exp_avg_sq": moments[n][1].clone()}
                 for i, n in enumerate(named)}
        return {"state": state if self.step_count else {},
                "param_groups": [{"lr": self.lr, "betas": self.betas, "eps": self.eps,
                                  "weight_decay": self.weight_decay, "amsgrad": False,
                                  "params": list(range(len(named)))}]}

    def check_errors(self) -> None:
        hip_ops.check_index_error(self.err)

    # --------------------------------------------------------------------- buffers ---
    def _buffers(self, B: int, F: int) -> _FFMBufs:
        b = self._bufsets.get((B, F))
        if b is None:
            dev, K = self.device, self.K
            S2, S = B * F * (F - 1), B * F
            e = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
            b = _FFMBufs(B=B, keys=torch.empty(max(S2, 1), dtype=torch.int32, device=dev),
                         vals=e(max(S2, 1), K), plan=hip_ops.SparsePlanBuffers(S2, dev),
                         plan_x=hip_ops.SparsePlanBuffers(S, dev), grad_rows=e(max(S2, 1), K),
                         slot_g=e(max(S, 1), 1), grad_w=e(max(S, 1), 1),
                         fwd=dict(z=e(B), p=e(B), loss_elem=e(B), gz=e(B)), loss=e(1))
            self._bufsets[(B, F)] = b
        self._bufs = b
        return b

    # ------------------------------------------------------------------------ step ----
    def step(self, x: torch.Tensor, y: torch.Tensor, return_loss: bool = True):
        """One training step on batch (x [B,F] int64/int32, y [B] 0/1); returns the mean
        BCE as a fresh 1-element device tensor (no host sync), or None with
        return_loss=False. Every step adds its loss to ``loss_sum`` (float64, on the device;
        read_loss_sum / reset_loss_sum, as FusedCTRTrainer)."""
        with self._scratch.scope():
            loss = self._step(x, y)
            return loss.clone() if return_loss else None

    def reset_loss_sum(self) -> None:
        self.loss_sum.zero_()

    def read_loss_sum(self) -> float:
        return float(self.loss_sum.item())

    def _step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        B, F = x.shape
        if F != self.F:
            raise ValueError(f"FusedFFMTrainer: batch has {F} fields, model {self.F}")
        if self._flush_due():
            self.flush()
        if self.use_graphs:
            return self._graph_step(x, y)
        self.step_table.ensure(self.step_count + 1)
        loss = self._launch(x, y)
        self._after_step()
        return loss

    def _flush_due(self) -> bool:
        """True when `flush_every` steps have passed since the last flush."""
        return self.flush_every > 0 and self.step_count - self._flushed_at >= self.flush_every

    def _after_step(self) -> None:
        self.step_count += 1
        self._dirty = True

    def _graph_step(self, x, y):
        if self.step_table.capacity < self.step_count + 2:
            self.step_table.ensure(max(self.step_count + 2, 2 * self.step_table.capacity))
        if self._graph_tab_version != self.step_table.version:
            torch.cuda.synchronize(self.device)  # none may still run when destroyed
            self._graphs.clear()  # they hold the old table's address
            self._graph_tab_version = self.step_table.version
        B, F = x.shape
        key = (B, F, x.dtype)
        inp = self._inputs.get(key)
        if inp is None:
            inp = self._inputs[key] = (torch.empty(B, F, dtype=x.dtype, device=self.device),
                                       torch.empty(B, dtype=torch.float32, device=self.device))
        xs, ys = inp
        xs.copy_(x, non_blocking=True)
        ys.copy_(y.reshape(-1), non_blocking=True)
        hit = self._graphs.get(key)
        if hit is None:
            loss = self._launch(xs, ys)  # the real step; also sizes every buffer
            self._after_step()
            if len(self._graphs) < self.max_graphs:
                g = torch.cuda.CUDAGraph()
                with graph_capture(g, pool=live_pool(self), stream=self._capture_stream):
                    self._launch(xs, ys)  # captured, not executed
                self._graphs[key] = (g, self._bufs)
                self.captures += 1
            return loss
        g, self._bufs = hit
        g.replay()
        self._after_step()
        return self._bufs.loss

    def _launch(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """Enqueue one step; step-dependent values come from the device step counter."""
        B, F = x.shape
        V, K = self.V, self.K
        b = self._buffers(B, F)
        y = y.reshape(-1)
        if y.dtype != torch.float32:
            y = y.float()
        y = y.contiguous()
        tabs = [e.weight.data for e in self.model.field_feature_embeddings]
        hint = self.step_count + 1
        opt = dict(betas=self.betas, eps=self.eps, weight_decay=self.weight_decay)
        # the batch's rows: plans over the (table, row) keys and over the ids
        hip_ops.ffm_keys(x, V, out=b.keys, err_flag=self.err)
        b.plan.build(b.keys[:b.plan.capacity], F * V)
        b.plan_x.build(x, V, err_flag=self.err)
        # catch-up: those rows replay the steps they missed (read the completed step)
        hip_ops.adam_deferred_rows(*self._table_args(), b.plan, hint, self.step_table, **opt,
                                   step_dev=self.step_done)
        hip_ops.adam_deferred_rows(*self._w_args(), b.plan_x, hint, self.step_table, **opt,
                                   step_dev=self.step_done)
        fwd = hip_ops.ffm_forward(x, tabs, self.ptrs, self.w, self.bias, labels=y, mean_div=B,
                                  err_flag=self.err, out=b.fwd)
        gz = fwd["gz"]
        hip_ops.ffm_backward(x, tabs, self.ptrs, gz, keys=b.keys, vals=b.vals)
        S2 = b.plan.capacity
        apply = dict(step_dev=self.step_cur, step_table=self.step_table, step=hint, **opt)
        if self._vec_ok and self.fuse_apply and K >= 32:
            hip_ops.segment_sum_rows_adam(b.plan, b.vals[:S2], None, self._table_args(), **apply,
                                          out=b.grad_rows, keep_sums=self.keep_grads)
        else:
            hip_ops.segment_sum_rows(b.plan, b.vals[:S2], out=b.grad_rows)
            hip_ops.adam_deferred_rows(*self._table_args(), b.plan, hint, self.step_table, **opt,
                                       grad_rows=b.grad_rows, step_dev=self.step_cur)
        # linear table: dL/dw[x_bf] = gz[b], summed per row in slot order
        b.slot_g.view(B, F).copy_(gz.view(B, 1).expand(B, F))
        hip_ops.segment_sum_rows(b.plan_x, b.slot_g[:B * F], out=b.grad_w)
        hip_ops.adam_deferred_rows(*self._w_args(), b.plan_x, hint, self.step_table, **opt,
                                   grad_rows=b.grad_w, step_dev=self.step_cur)
        hip_ops.tensor_sum(gz, out=self.g_bias)
        hip_ops.adam_dense(self.bias, self.g_bias, self.m_b, self.v_b, hint, self.lr,
                           self.betas, self.eps, self.weight_decay, step_dev=self.step_cur,
                           table=self.step_table)
        hip_ops.tensor_sum(fwd["loss_elem"], scale=1.0 / B, out=b.loss)
        hip_ops.step_end(self.step_ctr, b.loss, self.loss_sum)
        return b.loss
