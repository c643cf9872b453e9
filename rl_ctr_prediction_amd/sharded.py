"""Row-sharded data parallelism for the CTR step (BASELINE configs C3 at 8
GPUs and C5, the 40M-row table "sharded across 8xMI355X with RCCL all-to-all").

Rank r of N owns the embedding rows [r*Vs, (r+1)*Vs), Vs = ceil(V/N): their Adam moments,
their deferred-replay state and their updates. Every rank trains its own batch (weak
scaling); per step:

  1. sparse plan of the local batch (global ids); its unique rows are ascending, hence
     grouped by owner -> per-owner counts (ctr_plan_shard_counts), one tiny all-to-all of
     counts (the only host sync: variable-split collectives need sizes on the host);
  2. all-to-all of the unique row ids to their owners (each rank asks for each row once);
  3. owners bring the requested rows up to date (plan-free deferred catch-up: duplicates
     across requesters resolved by the owner scratch), gather E[row] and w[row] and send
     them back (all-to-all): every rank now holds its batch's rows compacted in unique order;
  4. forward + backward locally over that compact table (slot -> unique ordinal ids), the
     per-row gradient sums in plan order (the same kernels as the single-GPU step);
  5. all-to-all of the per-row gradients to the owners, which sum them per row in (source
     rank, position) order (a sparse plan over the received ids + the deterministic
     segmented sum) and apply Adam to their rows; the dense MLP gradient goes through one
     all-reduce as in the replicated path.

Per rank and step at C3 with 8 GPUs: ~61k unique rows out and back (ids 0.25 MB, rows and
gradients 16 MB each way) instead of all-gathering every rank's 16 MB of row gradients;
the deferred flush and the catch-up/apply work cover V/N rows. With N = 1 every exchange
is a local copy and the step is bitwise the single-GPU FusedCTRTrainer step
(tests/test_gpu_sharded.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import hip_ops
from .distributed import allreduce_sum_, alltoallv, exchange_counts, world
from .trainer import FusedCTRTrainer


class ShardedCTRTrainer(FusedCTRTrainer):
    """FusedCTRTrainer over this rank's row shard of the embedding tables (deferred-exact
    Adam). Rows outside the shard keep their initial values in this rank's copy of the
    model; gather_tables() assembles the trained tables."""

    def __init__(self, model, lr: float = 1e-3, weight_decay: float = 0.0, betas=(0.9, 0.999),
                 eps: float = 1e-8, process_group=None, seed: int | None = None,
                 count_group=None):
        """process_group: the ranks sharing the table (default: the world). count_group: a
        second communicator over the same ranks for the per-step counts exchange (it runs
        on the plan stream beside the data collectives). Default: created here with
        dist.new_group — a collective over the WHOLE world, so with the default
        process_group every rank builds its trainer at the same point; trainers over a
        sub-group must pass a count_group that every rank of the world created in the same
        order (e.g. one of dist.new_subgroups())."""
        self.rank, self.world_size = world()
        V = model.feature_embedding.weight.shape[0]
        if V < self.world_size:
            raise ValueError(f"row sharding: vocabulary {V} smaller than world size")
        self.shard_rows = -(-V // self.world_size)
        super().__init__(model, lr=lr, weight_decay=weight_decay, betas=betas, eps=eps,
                         process_group=process_group, seed=seed, optimizer_mode="deferred")
        if not self._vec_ok:
            raise ValueError("row sharding needs K % 4 == 0 and (K/4) dividing 64")
        self._side = None  # the exchange needs the plan before anything else
        self._slot2u = None
        self._counts = torch.zeros(self.world_size, dtype=torch.int64, device=self.device)
        # the plan and its per-owner counts are built on the plan stream (ahead of the step
        # with next_x), and the counts all-to-all — the step's one host sync — runs there on
        # a communicator of its own: the host then waits for the plan only, never for the
        # previous step's kernels or collectives, and runs ahead of the GPU
        if self._plan_stream is None:
            self._plan_stream = torch.cuda.Stream(device=self.device)
        self._count_group = count_group
        if self.world_size > 1 and count_group is None:
            if process_group is not None:
                raise ValueError("ShardedCTRTrainer over a process_group needs a count_group "
                                 "over the same ranks, created by every rank of the world "
                                 "(dist.new_group is collective over the whole world)")
            self._count_group = dist.new_group()
        self._ahead_counts: dict = {}
        # lookahead plans per ids tensor (LRU): ids key -> plan buffers / pending event
        self._plans: dict = {}
        self._pending: dict = {}
        self.max_plans = 16

    def _plan_for(self, x) -> hip_ops.SparsePlanBuffers:
        """The lookahead plan buffers of ids tensor x (least recently used reused first,
        never one still pending)."""
        key = self._xkey(x)
        p = self._plans.pop(key, None)
        if p is None:
            S = x.shape[0] * x.shape[1]
            if len(self._plans) >= self.max_plans:
                for k in list(self._plans):
                    if k not in self._pending:
                        old = self._plans.pop(k)
                        if old.capacity >= S:
                            p = old
                        break
            if p is None:
                p = hip_ops.SparsePlanBuffers(S, self.device)
        self._plans[key] = p  # most recently used last
        return p

    def _buffers(self, B: int, F: int):
        b = super()._buffers(B, F)
        if b.gplan is None:  # world size 1: the owner-side plan is still needed
            S = B * F * self.world_size
            e = lambda *s: torch.empty(*s, dtype=torch.float32, device=self.device)  # noqa: E731
            b.gplan = hip_ops.SparsePlanBuffers(S, self.device)
            b.g_rows, b.g_lin = e(S, self.K), e(S)
        return b

    def _table_rows(self) -> tuple[int, int]:
        lo = min(self.rank * self.shard_rows, self.V)
        return lo, min(lo + self.shard_rows, self.V)

    def step(self, x: torch.Tensor, y: torch.Tensor, global_batch: int | None = None,
             next_x=None) -> torch.Tensor:
        """next_x (one tensor or a sequence, as FusedCTRTrainer.step): the next batches'
        plans and per-owner counts are built on the plan stream during this step. Purely
        local (no collective depends on it), so ranks may pass different next_x."""
        B, F = x.shape
        ws = self.world_size
        mean_div = float(global_batch if global_batch is not None else B * ws)
        b = self._buffers(B, F)
        if self._slot2u is None or self._slot2u.numel() < B * F:
            self._slot2u = torch.empty(B * F, dtype=torch.int32, device=self.device)
        y = y.reshape(-1)
        if y.dtype != torch.float32:
            y = y.float()
        y = y.contiguous()
        bias, gv = self.views.get("bias"), self.grad_views
        has_lin = self.w_tab is not None  # InnerPNN: no linear table

        self._sync_weight_planes()
        self._bound_staleness()
        main, ps = torch.cuda.current_stream(), self._plan_stream
        xkey = self._xkey(x)
        ahead = [] if next_x is None else (
            [next_x] if isinstance(next_x, torch.Tensor) else list(next_x))
        ahead = [n for n in ahead if n.is_cuda and n.dim() == 2 and n.shape[1] == F
                 and self._xkey(n) != xkey]
        ev_start = torch.cuda.Event()
        ev_start.record(main)  # everything before this step (earlier readers of the plans)
        # 1. plan of the local batch, per-owner counts of its unique rows (plan stream)
        t = self._mark("plan")
        keep = {self._xkey(n) for n in ahead} | {xkey}
        for k in [k for k in self._pending if k not in keep]:
            del self._pending[k]
            self._ahead_counts.pop(k, None)
        if self._pending.pop(xkey, None) is not None:  # built ahead (ps is in order)
            plan, counts = self._plan_for(x), self._ahead_counts.pop(xkey)
        else:
            plan, counts = b.plan_own, self._counts
            ps.wait_event(ev_start)
            x.record_stream(ps)
            with torch.cuda.stream(ps):
                plan.build(x, self.V, err_flag=self.err)
                plan.shard_counts(self.shard_rows, ws, out=counts)
        b.plan = plan
        with torch.cuda.stream(ps):
            send_c, recv_c = exchange_counts(counts, self._count_group)
            ev_plan = torch.cuda.Event()
            ev_plan.record(ps)
        main.wait_event(ev_plan)
        self._span("plan", t)
        # 2. unique row ids to their owners, as shard-local ids
        t = self._mark("exchange")
        req = alltoallv(plan.unique_rows, send_c, recv_c, self.group)
        hip_ops.ids_add_(req, -self.row_lo)
        self._span("exchange", t)
        # 3. owners: catch the rows up, send them back
        t = self._mark("adam")
        hip_ops.adam_deferred_catchup_ids(self.E_tab, self.m_E, self.v_E, self.w_tab, self.m_w,
                                          self.v_w, self.last, req, self.rowmap, self.step_done,
                                          self.step_table, self.step_count + 1, self.betas,
                                          self.eps, self.weight_decay)
        self._span("adam", t)
        self._fork_sweep()
        t = self._mark("exchange")
        rows = hip_ops.embedding_gather(self.E_tab, req)
        T = alltoallv(rows, recv_c, send_c, self.group)
        T_lin = None
        if has_lin:
            lin = hip_ops.embedding_gather(self.w_tab, req)
            T_lin = alltoallv(lin, recv_c, send_c, self.group).view(-1)
        self._span("exchange", t)
        # 4. forward + backward over the compact table
        ids = plan.slot_to_unique(out=self._slot2u)[:B * F].view(B, F)
        if self.kind == "FM":
            t = self._mark("gather")
            hip_ops.fm_forward(ids, T, T_lin, bias, want_sum=True, labels=y, mean_div=mean_div,
                               want_p=False, out=b.fm)
            self._span("gather", t)
            gz = b.fm.gz
        else:
            gz = self._deepfm_forward_backward(ids, y, b, T, T_lin, bias, mean_div)
        if self.kind == "FM":  # DeepFM: summed on the weight-gradient stream
            hip_ops.tensor_sum(gz, out=gv["bias"].view(1))
        t = self._mark("scatter")
        if self.kind == "IPNN":  # per-slot gradients (through the pair products) summed per row
            hip_ops.segment_sum_rows(plan, b.dslot, out=b.grad_rows)
        else:
            hip_ops.fm_embedding_grad(plan, F, T, gz, b.fm.sum_e, b.dx, None,
                                      grad_rows=b.grad_rows, grad_lin=b.grad_lin, compact=True)
        self._span("scatter", t)
        if self.kind != "FM":  # the dense-parameter gradients, on the weight-gradient stream
            self._weight_grads(b, gz)
        if self.kind == "FM":  # DeepFM: summed on the weight-gradient stream (joined below)
            hip_ops.tensor_sum(b.fm.loss_elem, scale=1.0 / B, out=b.loss)
        # 5. gradients to the owners, summed per row in (source rank, position) order
        t = self._mark("exchange")
        G = alltoallv(b.grad_rows, send_c, recv_c, self.group)
        G_lin = alltoallv(b.grad_lin, send_c, recv_c, self.group) if has_lin else None
        self._join_wgrad()
        allreduce_sum_(self.flat_grad, self.group)
        if ws > 1:
            allreduce_sum_(b.loss, self.group)
            b.loss.div_(ws)
        self._span("exchange", t)
        t = self._mark("scatter")
        b.gplan.build(req, self.V_tab)
        hip_ops.segment_sum_rows(b.gplan, G, G_lin, rowmap=None, out=b.g_rows,
                                 out_lin=b.g_lin if has_lin else None)
        self._span("scatter", t)
        self.step_count += 1
        t = self._mark("adam")
        hip_ops.adam_deferred_rows(self.E_tab, self.m_E, self.v_E, self.w_tab, self.m_w,
                                   self.v_w, self.last, b.gplan, self.step_count,
                                   self.step_table, self.betas, self.eps, self.weight_decay,
                                   grad_rows=b.g_rows, grad_lin=b.g_lin if has_lin else None,
                                   step_dev=self.step_cur)
        self._span("adam", t)
        self._dirty = True
        self._adam_dense(self.step_count)
        self._join_sweep()
        hip_ops.step_end(self.step_ctr)
        for n in ahead:  # the next batches' plans and counts, concurrent with this step
            k = self._xkey(n)
            if k in self._pending:
                continue
            P = self._plan_for(n)
            c = torch.empty(ws, dtype=torch.int64, device=self.device)
            ps.wait_event(ev_start)
            n.record_stream(ps)
            with torch.cuda.stream(ps):
                P.build(n, self.V, err_flag=self.err)
                P.shard_counts(self.shard_rows, ws, out=c)
                ev = torch.cuda.Event()
                ev.record(ps)
            self._pending[k] = ev
            self._ahead_counts[k] = c
        return b.loss

    def gather_tables(self) -> tuple[torch.Tensor, torch.Tensor | None]:
        """Full (E [V,K], w [V,1] or None for InnerPNN) assembled from every rank's shard
        (after a flush)."""
        self.flush()
        E = self.model.feature_embedding.weight.data
        w = self.model.linear.weight.data if self.w_tab is not None else None
        if self.world_size == 1:
            return E.clone(), (w.clone() if w is not None else None)

        def gather(tab, width):
            out = torch.empty(self.shard_rows * self.world_size, width, dtype=tab.dtype,
                              device=tab.device)
            send = torch.zeros(self.shard_rows, width, dtype=tab.dtype, device=tab.device)
            send[:self.V_tab] = tab.view(self.V_tab, width)
            if tab.is_cuda and dist.get_backend(self.group) == "gloo":
                o = out.cpu()
                dist.all_gather_into_tensor(o, send.cpu(), group=self.group)
                out.copy_(o)
            else:
                dist.all_gather_into_tensor(out, send, group=self.group)
            return out[:self.V]

        return gather(self.E_tab, self.K), (gather(self.w_tab, 1) if w is not None else None)
