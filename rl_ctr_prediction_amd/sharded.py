"""Row-sharded data parallelism for the CTR step (BASELINE configs C3 at 8
GPUs and C5, the 40M-row table "sharded across 8xMI355X with RCCL all-to-all").

Rank r of N owns the embedding rows [r*Vs, (r+1)*Vs), Vs = ceil(V/N): their values, Adam
moments, deferred-replay state and updates — and nothing else of the tables (the rank's
copy of the model holds its shard only). Every rank trains its own batch (weak scaling);
per step:

  1. sparse plan of the local batch (global ids), built on the plan stream (ahead of the
     step with next_x); its unique rows are ascending, hence grouped by owner;
  2. the exchange capacity C: the largest per-owner run over every rank's batch (one
     all-reduce MAX of a scalar on a capacity stream that waits for the batch's plan only,
     read by the host: the step's only host read, which never waits for the main stream's
     queued steps — with next_x the plan finished long before); the capacity in use only
     grows — past a batch that exceeds it, to that run + 1/32, rounded up to 1024 rows — so
     after the first few steps every batch fits one capacity (one set of buffers, one
     graph per input slot);
  3. equal-split all-to-alls of C rows per (requester, owner) pair — row ids out
     (ctr_shard_pack_ids: each owner's run, padded with the owner's spare row), rows back,
     gradients out (ctr_shard_runs_copy packs / unpacks the runs): their sizes depend on C
     alone, so the step has no variable-split collective and, for a given C, is one fixed
     launch sequence (captured as a HIP graph, RCCL collectives included; gloo: eager);
  4. owners bring the requested rows up to date (plan-free deferred catch-up: duplicates
     across requesters resolved by the owner scratch), gather E[row] and w[row] and send
     them back: every rank then holds its batch's rows compacted in unique order;
  5. forward + backward locally over that compact table (slot -> unique ordinal ids), the
     per-row gradient sums in plan order (the same kernels as the single-GPU step);
  6. the per-row gradients go to the owners, which sum them per row in (source rank,
     position) order — a sparse plan over the received ids + the deterministic segmented
     sum; padding entries form the spare row's segment, summed and applied to the spare
     row, which nothing reads — and apply Adam to their rows; the dense MLP gradient goes
     through one all-reduce.

Per rank and step at C3 with 8 GPUs: ~61k unique rows out and back (ids 0.25 MB, rows and
gradients 16 MB each way, plus the padding up to C) instead of all-gathering every rank's
16 MB of row gradients; the deferred flush and the catch-up / apply work cover V/N rows.
With N = 1 every exchange is a local copy and the step is bitwise the single-GPU
FusedCTRTrainer step (tests/test_gpu_sharded.py). exchange="varsplit" keeps the
variable-split protocol (per-owner counts all-to-all, sizes on the host) for comparison:
both give bitwise the same results.
"""
from __future__ import annotations

import os
import warnings
import weakref
from time import perf_counter

import torch
import torch.distributed as dist

from . import hip_ops
from .distributed import allreduce_sum_, alltoall_equal, alltoallv, exchange_counts, world
from .trainer import FusedCTRTrainer, InputSlot, graph_capture, live_pool

CAP_QUANTUM = 1024  # exchange capacities are multiples of this many rows


class _XBufs:
    """The fixed-capacity exchange buffers of one (batch shape, capacity). Rows travel with
    their linear weight in one chunk per (requester, owner) pair (hip_ops.rows_chunk floats:
    C rows of K, then the C weights), so each direction is one all-to-all."""

    def __init__(self, n: int, C: int, S: int, K: int, lin: bool, dev):
        i32 = dict(dtype=torch.int32, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        NC = n * C
        self.C = C
        self.chunk = hip_ops.rows_chunk(C, K, lin)
        self.send_ids, self.recv_ids = torch.empty(NC, **i32), torch.empty(NC, **i32)
        self.counts, self.offsets = torch.empty(n, **i32), torch.empty(n, **i32)
        # every chunk's C rows in source order: the owner's view of the received gradients
        self.all_counts = torch.full((n,), C, **i32)
        self.all_offsets = torch.arange(n, **i32) * C
        self.rows_out, self.rows_in = (torch.empty(n * self.chunk, **f32) for _ in range(2))
        self.g_out, self.g_recv = (torch.empty(n * self.chunk, **f32) for _ in range(2))
        self.table = torch.empty(max(S, 1), K, **f32)  # the batch's rows, compact
        self.g_in = torch.empty(NC, K, **f32)          # owner: received gradients, by source
        self.g_rows = torch.empty(NC, K, **f32)
        if lin:
            self.lin_table = torch.empty(max(S, 1), **f32)
            self.glin_in = torch.empty(NC, **f32)
            self.g_lin = torch.empty(NC, **f32)
        else:
            self.lin_table = self.glin_in = self.g_lin = None
        self.gplan = hip_ops.SparsePlanBuffers(NC, dev)


def _host_span(acc: dict, key: str, t0: float) -> float:
    t1 = perf_counter()
    acc[key] = acc.get(key, 0.0) + (t1 - t0)
    return t1


UNKNOWN_RUN = 1 << 62  # an agreement entry whose batch some rank has not staged (MAX wins)


class _Agreement:
    """One capacity agreement: the largest per-owner run of the batches each rank staged for
    the next LOOKAHEAD steps (entry j: step t + 1 + j; UNKNOWN_RUN where not staged), all-
    reduced MAX over the count group (N > 1), copied to pinned host memory, an event after."""

    __slots__ = ("dev", "host", "ev", "keys", "call")

    def __init__(self, n: int, dev):
        self.dev = torch.empty(n, dtype=torch.int64, device=dev)
        self.host = torch.empty(n, dtype=torch.int64, pin_memory=True)
        self.ev = torch.cuda.Event()
        # this rank's batch behind each entry: (ids key, staging generation of its slot), so
        # a slot re-staged after the agreement measured it is never sized by that agreement
        self.keys = [None] * n
        self.call = None        # the step() call that issued it


class ShardedCTRTrainer(FusedCTRTrainer):
    """FusedCTRTrainer over this rank's row shard of the embedding tables (deferred-exact
    Adam). The shard is all this rank keeps: at construction the model's
    ``feature_embedding.weight`` (and ``linear.weight``) data are replaced by rows
    [row_lo, row_hi) — copied to the device, the full table released — so a rank holds
    ceil(V/N) rows of E, w and their Adam state (+ one spare row, the exchange's padding
    target), never the whole table. The model may be built on the host (the reference's own
    init: ``get_model(...)`` then ``.to(device)``, all_main/pretrain_main.py:137), so a
    vocabulary larger than one GPU is never materialised on any device.
    ``model.state_dict()`` is local (no collective): this rank's rows of the tables (their
    row range in the dict's metadata) and the replicated dense parameters; every rank saves
    and resumes from its own file with ``model.load_state_dict`` (a full-size table in the
    loaded dict is cut to the rank's rows; another rank's shard is refused). full_state_dict() and
    gather_tables() — collectives, every rank calls them — assemble the full tables; the
    sharded model's own forward needs them and refuses to run on a shard (N > 1)."""

    LOOKAHEAD = 2  # steps ahead a capacity agreement covers

    def __init__(self, model, lr: float = 1e-3, weight_decay: float = 0.0, betas=(0.9, 0.999),
                 eps: float = 1e-8, process_group=None, seed: int | None = None,
                 count_group=None, device=None, exchange: str = "padded",
                 force_collectives: bool = False, layout: str | None = None):
        """process_group: the ranks sharing the table (default: the world). count_group: a
        second communicator over the same ranks for the per-step capacity / counts
        agreement (it runs on the plan stream beside the data collectives). Default:
        created here with dist.new_group — a collective over the WHOLE world, so with the
        default process_group every rank builds its trainer at the same point; trainers
        over a sub-group must pass a count_group that every rank of the world created in
        the same order (e.g. one of dist.new_subgroups()). exchange: "padded" (fixed
        capacity, the default) or "varsplit". force_collectives: at world size 1, send every
        exchange through the collectives of a one-rank process group (dist initialised,
        e.g. RCCL on one GPU) instead of local copies — the N > 1 launch sequence, RCCL
        kernels and their graph capture included, on one device (tests). layout: "cyclic"
        (the default; CTR_SHARD_LAYOUT overrides) — global row r lives on rank r % N as its
        local row r // N — or "blocks" — rank r owns the contiguous rows [r*Vs, (r+1)*Vs).
        The reference's encoders number the feature ids field by field (creat_data.py's field
        offsets), so the high-cardinality fields fill the last row blocks: measured on the
        Criteo-shape C3 batches at N = 8 (gloo rehearsal, profiles/r06_n8_rehearsal.jsonl),
        blocks gave one owner ~85 % of every batch's unique rows and an exchange capacity of
        41,984 rows per pair against ~7,600 rows per owner on average (82 % padding); cyclic
        ownership spreads every field over every rank."""
        self.rank, self.world_size = world()
        V = model.feature_embedding.weight.shape[0]
        if V < self.world_size:
            raise ValueError(f"row sharding: vocabulary {V} smaller than world size")
        if exchange not in ("padded", "varsplit"):
            raise ValueError(f"exchange must be 'padded' or 'varsplit', not {exchange!r}")
        self.exchange = exchange
        layout = layout or os.environ.get("CTR_SHARD_LAYOUT", "cyclic")
        if layout not in ("cyclic", "blocks"):
            raise ValueError(f"layout must be 'cyclic' or 'blocks', not {layout!r}")
        self.layout = layout
        self.shard_rows = -(-V // self.world_size)
        self._V_full = V
        # cyclic at N > 1: the batch ids are permuted (ctr_shard_permute_ids) into the space
        # where each rank's rows are one block again; at N = 1 both layouts are the identity
        self._permute = layout == "cyclic" and self.world_size > 1
        self._V_plan = self.shard_rows * self.world_size if self._permute else V
        self._shard_model(model, device)
        super().__init__(model, lr=lr, weight_decay=weight_decay, betas=betas, eps=eps,
                         process_group=process_group, seed=seed, optimizer_mode="deferred")
        if not self._vec_ok:
            raise ValueError("row sharding needs K % 4 == 0 and (K/4) dividing 64")
        self._side = None  # the exchange needs the plan before anything else
        self._pipe = False  # the dense gradient is all-reduced within its step
        # owners sum their received entries (<= N per row) straight and apply in one launch;
        # CTR_OWNER_DIRECT=0: the chunked segmented sums with the fused apply (A/B)
        self._owner_direct = os.environ.get("CTR_OWNER_DIRECT", "1") != "0"
        # requesters write their row sums straight into the exchange chunks (the padding rows
        # past each run are left unwritten: only the direct owner pass, which skips the spare
        # row they map to, may read them); CTR_GRADS_TO_CHUNKS=0: compact sums + pack (A/B)
        self._grads_to_chunks = (self._owner_direct and
                                 os.environ.get("CTR_GRADS_TO_CHUNKS", "1") != "0")
        self._slot2u = None
        self._counts = torch.zeros(self.world_size, dtype=torch.int64, device=self.device)
        # the plans (and per-owner counts / run maxima) are built on the plan stream, ahead
        # of the step with next_x; the capacity agreements run on a stream and (N > 1) a
        # communicator of their own (_capacity)
        if self._plan_stream is None:
            self._plan_stream = self._new_stream()
        self._count_group = count_group
        # collectives in the step: always at N > 1; at N = 1 only when forced
        self._coll = self.world_size > 1 or bool(force_collectives)
        if self._coll and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("force_collectives needs an initialised process group")
        if self._coll and count_group is None:
            if process_group is not None:
                raise ValueError("ShardedCTRTrainer over a process_group needs a count_group "
                                 "over the same ranks, created by every rank of the world "
                                 "(dist.new_group is collective over the whole world)")
            self._count_group = dist.new_group()
        self._ahead_counts: dict = {}
        # the capacity agreements (see _capacity): one per step() call, issued at the end of
        # the call for the batches staged for the next LOOKAHEAD steps, read back two calls
        # later at the latest; a ring of four (a record is reused four calls after its issue)
        self._cap_stream = self._new_stream()
        self._agree = [_Agreement(self.LOOKAHEAD, self.device) for _ in range(4)]
        self._calls = 0           # step() calls so far (the index of the next step)
        self._stage_gen = 0       # slot stagings so far (InputSlot.gen)
        self._plan_graphs_ok = True
        self._agree_last_ev = None
        self._now = None          # the blocking agreement's record (no lookahead)
        self.cap_reads = 0        # host reads of an agreement (one per step)
        self.cap_blocking = 0     # of those, agreements made in the step itself
        # host seconds per section of step() (tools/sharded_host_cost.py), when a dict
        self.host_sections: dict | None = None
        self._xbufs: dict = {}
        self._cap = 0  # the exchange capacity in use (rows per (requester, owner) pair)
        # graph replay of the fixed-capacity step: at one process always, at N > 1 where the
        # collectives can be captured — RCCL (nccl backend; round 5: the one-rank RCCL step
        # captured with its all_to_all_single / all_reduce kernels is bitwise the eager and
        # the local-copy step on the MI355X, test_rccl_world1_collectives_bitwise) — unless
        # CTR_SHARDED_GRAPHS=0; gloo stages through the host and cannot be captured
        backend = dist.get_backend(self.group) if self.world_size > 1 else None
        self._graph_ok = self.world_size == 1 or (
            backend == "nccl" and os.environ.get("CTR_SHARDED_GRAPHS", "1") != "0")
        # varsplit: lookahead plans per ids tensor (LRU): ids key -> plan buffers / event
        self._plans: dict = {}
        self._pending: dict = {}
        self.max_plans = 16

    # ----------------------------------------------------------------- the shard ------
    def _shard_model(self, model, device) -> None:
        """Replace the model's table data by this rank's rows on the device (before the
        base class reads the model) and move the rest of the model there. The rows live in
        a buffer with one spare row past the shard (the exchange's padding entries read and
        update it); the Parameter is the view of the real rows."""
        E = model.feature_embedding.weight
        if device is None:
            device = E.device if E.is_cuda else torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        n_r = self._rows_of(self.rank)
        tabs = [E] + ([model.linear.weight] if hasattr(model, "linear") else [])
        self._spare = {}
        for p in tabs:
            buf = torch.zeros((n_r + 1,) + tuple(p.shape[1:]), dtype=p.dtype, device=device)
            buf[:n_r].copy_(self._cut(p.data))  # the full table's storage goes with .data
            p.data = buf[:n_r]
            self._spare[id(p)] = buf
        model.to(device)
        self._sharded_params = tabs
        if E.device.type == "cuda" or device.type == "cuda":
            # the full table's device block goes back to the device, not to this process's
            # cache (ranks that share a GPU — the gloo rehearsal of N > 1 on one device —
            # would otherwise each hold a full table's worth of cached memory)
            torch.cuda.empty_cache()
        if self.world_size > 1:
            ref = weakref.ref(self)

            def no_forward(*_):
                raise RuntimeError("ShardedCTRTrainer: this model holds one row shard of its "
                                   "tables; assemble them with trainer.gather_tables() (or "
                                   "model.state_dict() on every rank) for inference")

            def save_rows(module, state_dict, prefix, local_metadata):
                """The shard's row range goes into the state dict's metadata (the keys stay
                the reference's): [row_lo, row_hi, V]."""
                t = ref()
                if t is not None:
                    local_metadata["ctr_rows"] = t.shard_meta()

            def load_rows(state_dict, prefix, local_metadata, strict, missing, unexpected,
                          errors):
                """A full-size table in the loaded dict (a checkpoint of the unsharded model
                or of full_state_dict()) is cut to this rank's rows; a shard-size one loads as
                it is only if its metadata names this rank's rows (a shard saved by another
                rank, or without its row range, is refused: equal shard sizes would otherwise
                load another rank's rows without an error)."""
                t = ref()
                if t is None:
                    return
                for name in ("feature_embedding.weight", "linear.weight"):
                    v = state_dict.get(prefix + name)
                    if v is None or v.dim() < 1:
                        continue
                    if v.shape[0] == t._V_full != t.V_tab:
                        state_dict[prefix + name] = t._cut(v)
                        continue
                    got = local_metadata.get("ctr_rows")
                    want = t.shard_meta()
                    if got is None or list(got) != want:
                        raise RuntimeError(
                            f"ShardedCTRTrainer: {prefix + name} holds {v.shape[0]} rows with "
                            f"row range {got} in its metadata; this rank owns the rows {want} "
                            "— load this rank's own state_dict() or a full-size table "
                            "(full_state_dict())")
            model.register_forward_pre_hook(no_forward)
            model._register_state_dict_hook(save_rows)
            model._register_load_state_dict_pre_hook(load_rows)

    def _vocab_size(self, E) -> int:
        return self._V_full

    def _rows_of(self, r: int) -> int:
        """Rows of the table rank r owns."""
        V, n = self._V_full, self.world_size
        if self.layout == "cyclic":
            return max(0, (V - r + n - 1) // n)
        lo = min(r * self.shard_rows, V)
        return min(lo + self.shard_rows, V) - lo

    def _cut(self, full: torch.Tensor, r: int | None = None) -> torch.Tensor:
        """Rank r's rows (default: this rank's) of a full-size table, in local order."""
        r = self.rank if r is None else r
        if self.layout == "cyclic":
            return full[r::self.world_size]
        lo = min(r * self.shard_rows, self._V_full)
        return full[lo:lo + self._rows_of(r)]

    def shard_meta(self) -> list:
        """The shard's identity as saved in the state dict's metadata ("ctr_rows"):
        ["cyclic", rank, N, V] or, for the blocks layout, [row_lo, row_hi, V]."""
        if self.layout == "cyclic":
            return ["cyclic", self.rank, self.world_size, self._V_full]
        lo = min(self.rank * self.shard_rows, self._V_full)
        return [lo, lo + self._rows_of(self.rank), self._V_full]

    def _plan_ids(self, x: torch.Tensor) -> torch.Tensor:
        """The ids the plans are built over: x itself, or (cyclic, N > 1) a permuted copy."""
        if not self._permute:
            return x
        xp = x.contiguous().clone() if x.is_cuda else x.to(self.device)
        return hip_ops.shard_permute_ids_(xp, self.V, self.world_size, self.shard_rows,
                                          err_flag=self.err)

    def _own_rows(self, t: torch.Tensor) -> torch.Tensor:
        """The shard's buffer, spare row included (the Parameter is its first V_tab rows)."""
        for p in self._sharded_params:
            if p.data.data_ptr() == t.data_ptr():
                buf = self._spare[id(p)]
                return buf.view(-1) if t.dim() == 2 and t.shape[1] == 1 else buf
        return t

    def _buffers(self, B: int, F: int):
        fresh = (B, F) not in self._bufsets
        b = super()._buffers(B, F)
        if fresh and self._coll and self.exchange == "padded":
            # the batch loss lives in the dense gradient's tail: one all-reduce carries both
            n = self.flat_grad.numel()
            b.loss = self._grad_ext[n:n + 1]
        if b.gplan is None:  # world size 1: the owner-side plan is still needed
            S = B * F * self.world_size
            e = lambda *s: torch.empty(*s, dtype=torch.float32, device=self.device)  # noqa: E731
            b.gplan = hip_ops.SparsePlanBuffers(S, self.device)
            b.g_rows, b.g_lin = e(S, self.K), e(S)
        return b

    def _table_rows(self) -> tuple[int, int]:
        """The rank's rows as a range of the plan's id space (the permuted one, cyclic N > 1):
        [rank * Vs, rank * Vs + rows)."""
        lo = self.rank * self.shard_rows if self._permute else min(self.rank * self.shard_rows,
                                                                   self.V)
        return lo, lo + self._rows_of(self.rank)

    def optimizer_state_dict(self) -> dict:
        """The shard's moments (the spare row is internal): only the table parameters'
        entries are trimmed, picked by name — a dense parameter whose length happens to be
        V_tab + 1 keeps every element."""
        st = super().optimizer_state_dict()
        names = [n for n, _ in self.model.named_parameters()]
        for i, s in st["state"].items():
            if names[i] in ("feature_embedding.weight", "linear.weight"):
                for k in ("exp_avg", "exp_avg_sq"):
                    s[k] = s[k][:self.V_tab]
        return st

    def full_state_dict(self, device=None) -> dict:
        """model.state_dict() with the full tables assembled from every rank's shard — a
        collective: EVERY rank calls it (device="cpu" for a table larger than one GPU)."""
        sd = self.model.state_dict()
        E_full, w_full = self.gather_tables(device=device)
        sd["feature_embedding.weight"] = E_full
        if w_full is not None:
            sd["linear.weight"] = w_full.view(-1, 1)
        return sd

    # ------------------------------------------------------------------ the step ------
    def _step(self, x: torch.Tensor, y: torch.Tensor, global_batch: int | None = None,
              next_x=None, next_y=None) -> torch.Tensor:
        """next_x (one tensor or a sequence, as FusedCTRTrainer.step): the batches of the next
        steps, in step order. They are staged and their plans and per-owner run maxima built
        on the plan stream during this step, and the capacity for the next LOOKAHEAD steps is
        agreed at the end of this call (_capacity). At N > 1 a batch passed as next_x[j]
        must be the batch of step + 1 + j once that step comes (the ranks agreed on its
        capacity; any rank may pass None or fewer batches, and every rank then agrees in
        the step instead). next_y is accepted and not used here (the labels are copied with
        each step)."""
        if self.exchange == "varsplit":
            return self._step_varsplit(x, y, global_batch, next_x)
        hs = self.host_sections
        h0 = perf_counter() if hs is not None else 0.0
        B, F = x.shape
        ws = self.world_size
        mean_div = float(global_batch if global_batch is not None else B * ws)
        self._sync_weight_planes()
        self._bound_staleness()
        main, ps = hip_ops.current_stream(), self._plan_stream
        shape = (B, F, x.dtype)
        xkey = self._xkey(x)
        t_call = self._calls
        # the next batches by position (entry j: step t_call + 1 + j); None where a batch
        # cannot be staged (another shape, the current batch, a repeat)
        ahead = []
        if next_x is not None:
            for n in ([next_x] if isinstance(next_x, torch.Tensor) else next_x):
                k = self._xkey(n)
                ok = (k[1:3] == xkey[1:3] and k != xkey
                      and all(a is None or k != a[1] for a in ahead))
                ahead.append((n, k) if ok else None)
        slot = self._staged.pop(xkey, None)
        if self._staged:
            # batches staged ahead stay staged while next_x names them or an agreement
            # already issued covers them (call t-1's entry for step t+1): their plans are
            # what those agreements measured
            keep = {a[1] for a in ahead if a is not None} | self._agreed_keys(t_call)
            for k in [k for k in self._staged if k not in keep]:
                main.wait_event(self._staged.pop(k).ev)
        todo = [a for a in ahead if a is not None and a[1] not in self._staged]
        ev_start = self._start_event()
        ev_start.record(main)  # everything enqueued before this step
        if slot is None:  # copy and plan now, on the plan stream
            slot = self._acquire_slot(shape, ahead=True)
            self._stage_slot(slot, x, ev_start, main)
        slot.y.copy_(y.reshape(-1), non_blocking=True)
        if hs is not None:
            h0 = _host_span(hs, "prologue", h0)
        t = self._mark("plan")
        cmax = self._capacity(t_call, xkey, slot)
        self._span("plan", t)
        if hs is not None:
            h0 = _host_span(hs, "capacity_read", h0)
        if cmax > self._cap:  # grows only (every rank sees the same cmax: the same C)
            grown = cmax + cmax // 32  # headroom: a later, slightly larger batch still fits
            C = max(CAP_QUANTUM, -(-grown // CAP_QUANTUM) * CAP_QUANTUM)
            if self._xbufs:  # the smaller capacity's buffers and graphs are never used again
                torch.cuda.synchronize(self.device)
                self._graphs = {k: v for k, v in self._graphs.items() if k[2] == C}
                self._xbufs = {k: v for k, v in self._xbufs.items() if k[2] == C}
            self._cap = C
        C = self._cap
        main.wait_event(slot.ev)  # the slot's ids copy, plan and per-owner runs
        if self.use_graphs and self._graph_ok and self.timing is None:
            loss = self._sharded_graph_step(slot, mean_div, C)
        else:
            self.step_table.ensure(self.step_count + 1)
            loss = self._launch_sharded(slot, mean_div, C)
            self._after_step()
        if hs is not None:
            h0 = _host_span(hs, "step_launch", h0)
        for n, k in todo:
            s = self._acquire_slot(shape, exclude=slot, ahead=True)
            self._stage_slot(s, n, ev_start, main)
            self._staged[k] = s
        if hs is not None:
            h0 = _host_span(hs, "stage_ahead", h0)
        self._issue_agreement(t_call, ahead)
        self._calls += 1
        if hs is not None:
            _host_span(hs, "agreement_issue", h0)
        return loss

    # ----------------------------------------------------------- the capacity ---------
    # The step's one host read is the exchange capacity C: every rank's largest per-owner
    # run, agreed before the step's collectives can be sized. Where the read is enqueued
    # decides what it waits for: a process has GPU_MAX_HW_QUEUES (4) hardware queues and the
    # HIP runtime maps every further stream onto one of them (least used at creation), so a
    # stream of its own is no guarantee that a read does not queue behind the main stream's
    # steps (round 4: the capacity stream landed on the plan stream's queue in one process
    # and, in the test suite's process with more streams created before, on main's). So the
    # agreement for a step is enqueued in an EARLIER call: at the end of call t (after its
    # step and staging), for the batches staged for steps t+1 and t+2; the read at step t
    # takes the agreement of call t-2 (entry 1) or else of call t-1 (entry 0). In FIFO order
    # on whatever queue it lands, that agreement sits behind at most the work enqueued up to
    # call t-1's end — never behind anything enqueued after (test_capacity_read_never_waits_
    # for_main: a sleep kernel queued on main between two calls). With two batches of
    # lookahead the read waits for step t-2 at worst, so the host runs up to two steps ahead
    # of the GPU. A step whose capacity nobody agreed ahead (no lookahead on some rank: every
    # rank sees the same UNKNOWN_RUN) agrees in the step itself (_agree_now).

    def _agreed_keys(self, t: int) -> set:
        """The ids keys of the batches an issued agreement covers beyond step t (call t-1's
        entries past step t)."""
        a = self._agree[(t - 1) % 4]
        if a.call != t - 1:
            return set()
        return {k[0] for k in a.keys[1:] if k is not None}

    def _capacity(self, t: int, xkey, slot: InputSlot) -> int:
        """The agreed capacity need (largest run) of step t."""
        for a, j in ((self._agree[(t - 2) % 4], 1), (self._agree[(t - 1) % 4], 0)):
            if a.call != t - 1 - j or j >= len(a.keys):
                continue
            a.ev.synchronize()
            v = int(a.host[j])
            if v == UNKNOWN_RUN:
                continue
            key = a.keys[j]
            if key is not None and key == (xkey, slot.gen):
                self.cap_reads += 1
                return v
            if self._coll:  # the other ranks sized this step by that agreement
                what = ("a batch re-staged after its capacity was agreed (the slot the "
                        "agreement measured was dropped)" if key is not None and key[0] == xkey
                        else "a batch other than the one passed as next_x for it")
                raise RuntimeError(
                    f"ShardedCTRTrainer: step trained on {what}; with collectives every rank "
                    "sized this step's exchange by the agreed capacity of the announced "
                    "batches (pass next_x=None instead)")
            break  # one process: agree on this batch now
        return self._agree_now(slot)

    def _agree_now(self, slot: InputSlot) -> int:
        """The capacity of this step's batch alone, agreed now (blocking)."""
        a = self._now
        if a is None:
            a = self._now = _Agreement(1, self.device)
        cs, main = self._cap_stream, hip_ops.current_stream()
        cs.wait_event(slot.ev)
        torch.cuda.set_stream(cs)
        try:
            a.dev.copy_(slot.cap)
            if self._coll:
                dist.all_reduce(a.dev, op=dist.ReduceOp.MAX, group=self._count_group)
            a.host.copy_(a.dev, non_blocking=True)
            a.ev.record(cs)
        finally:
            torch.cuda.set_stream(main)
        a.ev.synchronize()
        self.cap_reads += 1
        self.cap_blocking += 1
        return int(a.host[0])

    def _issue_agreement(self, t: int, ahead) -> None:
        """Call t's agreement for steps t+1 .. t+LOOKAHEAD (not waited for here)."""
        a = self._agree[t % 4]
        a.call = t
        cs = self._cap_stream
        known = []
        for j in range(self.LOOKAHEAD):
            e = ahead[j] if j < len(ahead) else None
            s = self._staged.get(e[1]) if e is not None else None
            a.keys[j] = (e[1], s.gen) if s is not None else None
            if s is not None:
                cs.wait_event(s.ev)
                known.append((j, s))
        main = hip_ops.current_stream()
        torch.cuda.set_stream(cs)
        try:
            if len(known) < self.LOOKAHEAD:
                a.dev.fill_(UNKNOWN_RUN)
            for j, s in known:
                a.dev[j:j + 1].copy_(s.cap)
            if self._coll:
                dist.all_reduce(a.dev, op=dist.ReduceOp.MAX, group=self._count_group)
            a.host.copy_(a.dev, non_blocking=True)
            a.ev.record(cs)
        finally:
            torch.cuda.set_stream(main)
        self._agree_last_ev = a.ev

    def _stage_slot(self, s: InputSlot, ids: torch.Tensor, ev_start, main) -> None:
        """On the plan stream, after everything enqueued before this step and after the last
        agreement (which reads staged slots' run maxima): ids into slot s, its plan."""
        ps = self._plan_stream
        self._stage_gen += 1
        s.gen = self._stage_gen
        ps.wait_event(ev_start)
        if self._agree_last_ev is not None:
            ps.wait_event(self._agree_last_ev)
        torch.cuda.set_stream(ps)
        try:
            if not hip_ops.batch_stage_copy(s.ids, ids):
                s.ids.copy_(ids, non_blocking=True)
            if ids.is_cuda:
                ids.record_stream(ps)
            self._plan_slot(s)
        finally:
            torch.cuda.set_stream(main)

    def _slot_stream(self, stream_i: int):
        return self._plan_stream  # every slot is copied and planned on the one plan stream

    def _plan_slot(self, slot: InputSlot) -> None:
        """On the current (plan) stream: the slot's plan, its largest per-owner run
        (slot.cap, int64 scalar) and an event. Replayed from the slot's own captured graph
        once it exists (graphs on, no timing)."""
        if slot.cap is None:
            slot.cap = torch.zeros(1, dtype=torch.int64, device=self.device)
            slot.counts = torch.zeros(self.world_size, dtype=torch.int64, device=self.device)
            slot.slot2u = torch.empty(max(slot.ids.numel(), 1), dtype=torch.int32,
                                      device=self.device)
        if slot.plan_graph is not None and self.timing is None:
            slot.plan_graph.replay()
        else:
            self._plan_launch(slot)
            if self.use_graphs and self.timing is None and self._plan_graphs_ok:
                g = torch.cuda.CUDAGraph()
                # with collectives the process group's watchdog thread queries its events
                # while this thread captures: a thread-local capture, as the step's
                mode = "thread_local" if self._coll else "global"
                try:
                    with graph_capture(g, pool=live_pool(self), stream=hip_ops.current_stream(),
                                       capture_error_mode=mode):
                        self._plan_launch(slot)  # captured, not executed
                except RuntimeError as e:
                    if not self._coll:
                        raise
                    warnings.warn(f"ShardedCTRTrainer: plan graph capture failed ({e}); "
                                  "building the plans eagerly")
                    torch.cuda.synchronize(self.device)
                    self._plan_graphs_ok = False
                else:
                    slot.plan_graph = g
        slot.ev = self._slot_event(slot)
        slot.ev.record()

    def _plan_launch(self, slot: InputSlot) -> None:
        if self._permute:  # cyclic rows: the slot's ids into the per-owner block space
            hip_ops.shard_permute_ids_(slot.ids, self.V, self.world_size, self.shard_rows,
                                       err_flag=self.err)
        slot.plan.build(slot.ids, self._V_plan, err_flag=self.err)
        # the forward's ids over the compact table, ahead with the plan (off the step's path)
        slot.plan.slot_to_unique(out=slot.slot2u)
        if self.world_size <= 15:  # the counts and their maximum in one launch
            slot.plan.shard_counts(self.shard_rows, self.world_size, out=slot.counts,
                                   max_out=slot.cap)
        else:
            slot.plan.shard_counts(self.shard_rows, self.world_size, out=slot.counts)
            torch.amax(slot.counts, dim=0, keepdim=True, out=slot.cap)

    def _runs_mask(self, n_rows: int) -> torch.Tensor:
        """The owner plan's per-row run mask (zero between uses; ctr_sparse_plan_build_runs)."""
        m = getattr(self, "_rmask", None)
        if m is None or m.numel() < (n_rows + 3) // 4:
            m = self._rmask = torch.zeros((n_rows + 3) // 4, dtype=torch.int32,
                                          device=self.device)
        return m

    def _xb(self, B: int, F: int, C: int) -> _XBufs:
        key = (B, F, C)
        xb = self._xbufs.get(key)
        if xb is None:
            xb = self._xbufs[key] = _XBufs(self.world_size, C, B * F, self.K,
                                           self.w_tab is not None, self.device)
        return xb

    def _sharded_graph_step(self, slot: InputSlot, mean_div: float, C: int):
        if self.step_table.capacity < self.step_count + 2:
            self.step_table.ensure(max(self.step_count + 2, 2 * self.step_table.capacity))
        if self._graph_tab_version != self.step_table.version:
            torch.cuda.synchronize(self.device)
            self._graphs.clear()
            self._graph_tab_version = self.step_table.version
        mlp = getattr(self.model, "mlp", None)
        drops = tuple(float(mlp[i].p) for i in (2, 5)) if mlp is not None else ()
        key = (slot.shape, slot.index, C, mean_div, self.model.training, drops)
        hit = self._graphs.get(key)
        if hit is None:
            loss = self._launch_sharded(slot, mean_div, C)
            self._after_step()
            if len(self._graphs) < self.max_graphs:
                g = torch.cuda.CUDAGraph()
                # collectives inside: a thread-local capture, so the process group's
                # watchdog thread may query its events while this thread captures
                mode = "thread_local" if self._coll else "global"
                try:
                    with graph_capture(g, pool=live_pool(self), stream=self._capture_stream,
                                       capture_error_mode=mode):
                        self._launch_sharded(slot, mean_div, C)  # captured, not executed
                except RuntimeError as e:  # a backend that refuses capture: eager from here
                    if self.world_size == 1 and not self._coll:
                        raise
                    warnings.warn(f"ShardedCTRTrainer: step graph capture failed ({e}); "
                                  "launching the steps eagerly")
                    torch.cuda.synchronize(self.device)
                    self._graph_ok = False
                    return loss
                self._graphs[key] = (g, self._bufs)
                self.captures += 1
            return loss
        g, self._bufs = hit
        self._bufs.plan = slot.plan
        g.replay()
        self._after_step()
        return self._bufs.loss

    def _xchg(self, out: torch.Tensor, send: torch.Tensor, coll: bool) -> torch.Tensor:
        """The equal-split all-to-all of one exchange buffer into `out`, or (one process, no
        forced collectives) `send` itself: a one-rank all-to-all is the identity, so the
        readers take the send buffer and no copy is launched."""
        if not coll:
            return send
        alltoall_equal(out, send, self.group, force=True)
        return out

    def _launch_sharded(self, slot: InputSlot, mean_div: float, C: int) -> torch.Tensor:
        """Enqueue one fixed-capacity step (no host read, no size taken from the device:
        capturable for a given C)."""
        x, y = slot.ids, slot.y
        B, F = x.shape
        n = self.world_size
        f = self._coll  # the collectives (N > 1, or forced on a one-rank group)
        b = self._buffers(B, F)
        b.plan = plan = slot.plan
        xb = self._xb(B, F, C)
        bias, gv = self.views.get("bias"), self.grad_views
        has_lin = self.w_tab is not None
        step_hint = self.step_count + 1
        Vo = self.E_tab.shape[0]  # the owner's rows, spare row included
        # 1. row ids out: each owner's run, padded with its spare row
        t = self._mark("exchange")
        hip_ops.shard_pack_ids(plan, self.shard_rows, self.V, n, C, xb.send_ids, xb.counts,
                               xb.offsets, err_flag=self.err, cyclic=self._permute)
        recv_ids = self._xchg(xb.recv_ids, xb.send_ids, f)
        self._span("exchange", t)
        # 2. owners: the plan over the requested rows (every source's run, ascending, the
        # spare row as padding: ctr_sparse_plan_build_runs, 5 short launches instead of an
        # LSD sort's 8) — built here, ahead of the catch-up, which then runs over its
        # unique rows (one launch; the id-driven catch-up with its owner-marking pass took
        # 86 us at C3 against 24), and reused for the gradient sums of step 4 — then catch
        # the rows up, gather them, send them back
        t = self._mark("plan")
        if n <= 8:  # n ascending runs of unique rows + spare-row padding: the runs plan
            xb.gplan.build_runs(recv_ids, n, Vo, self._runs_mask(Vo))
        else:
            xb.gplan.build(recv_ids, Vo)
        self._span("plan", t)
        t = self._mark("catchup")
        hip_ops.adam_deferred_rows(self.E_tab, self.m_E, self.v_E, self.w_tab, self.m_w,
                                   self.v_w, self.last, xb.gplan, step_hint, self.step_table,
                                   self.betas, self.eps, self.weight_decay,
                                   step_dev=self.step_done)
        self._span("catchup", t)
        t = self._mark("exchange")
        # the rows and their linear weights: one gather, one all-to-all, one unpack
        hip_ops.shard_gather_rows(self.E_tab, self.w_tab if has_lin else None, recv_ids, n,
                                  C, out=xb.rows_out)
        rows_in = self._xchg(xb.rows_in, xb.rows_out, f)
        hip_ops.shard_rows_unpack(rows_in, C, xb.counts, xb.offsets, xb.table,
                                  xb.lin_table if has_lin else None)
        T_lin = xb.lin_table.view(-1, 1) if has_lin else None
        self._span("exchange", t)
        # 3. forward + backward over the compact table
        ids = slot.slot2u[:B * F].view(B, F)  # built with the slot's plan (_plan_launch)
        T = xb.table
        self._xb_cur = xb  # the row sums go straight into xb.g_out's chunks (_sharded_fwd_bwd)
        try:
            gz = self._sharded_fwd_bwd(ids, y, b, T, T_lin, bias, mean_div, F)
        finally:
            self._xb_cur = None
        # 4. gradients (with the linear ones) to the owners in one all-to-all, then every
        # source's chunk into the (source, position) order the owner plan indexes
        t = self._mark("exchange")
        if not self._grads_to_chunks or self.keep_grads:  # keep_grads: the compact sums stay
            hip_ops.shard_rows_pack(b.grad_rows, b.grad_lin if has_lin else None, C, xb.counts,
                                    xb.offsets, out=xb.g_out)
        g_recv = self._xchg(xb.g_recv, xb.g_out, f)
        if not self._owner_direct:  # the owners' chunked sums read (source, position) rows
            hip_ops.shard_rows_unpack(g_recv, C, xb.all_counts, xb.all_offsets, xb.g_in,
                                      xb.glin_in if has_lin else None)
        self._span("exchange", t)
        # 5. the owners' sums and Adam here, beside the weight-gradient stream (dW0 ...);
        # only the dense all-reduce and the dense Adam wait for it (6.)
        if self._owner_direct:
            # each row's <= N received entries summed straight in its lane group, then its
            # deferred Adam step, one launch (ctr_adam_deferred_entries); the spare row (the
            # padding target) is skipped
            t = self._mark("scatter")
            hip_ops.adam_deferred_entries(self.E_tab, self.m_E, self.v_E, self.w_tab, self.m_w,
                                          self.v_w, self.last, xb.gplan, g_recv, None,
                                          step_hint,
                                          self.step_table, self.betas, self.eps,
                                          self.weight_decay, skip_row=Vo - 1,
                                          step_dev=self.step_cur,
                                          out=xb.g_rows if self.keep_grads else None,
                                          out_lin=xb.g_lin if self.keep_grads and has_lin
                                          else None, run_len=C)
            self._span("scatter", t)
        elif self.fuse_apply and self.K >= self.fuse_apply_min_k:
            # the owners' row sums with each row's deferred Adam step applied where its sum
            # completes (ctr_segment_sum_rows_adam; bitwise the two passes below: one pass
            # over the rows instead of a sums write + read, N = 1 C3 29 us less)
            t = self._mark("scatter")
            table = (self.E_tab, self.m_E, self.v_E, self.w_tab, self.m_w, self.v_w, self.last)
            hip_ops.segment_sum_rows_adam(xb.gplan, xb.g_in, xb.glin_in if has_lin else None,
                                          table, step_dev=self.step_cur,
                                          step_table=self.step_table, step=step_hint,
                                          betas=self.betas, eps=self.eps,
                                          weight_decay=self.weight_decay, out=xb.g_rows,
                                          out_lin=xb.g_lin if has_lin else None,
                                          keep_sums=self.keep_grads)
            self._span("scatter", t)
        else:
            t = self._mark("scatter")
            hip_ops.segment_sum_rows(xb.gplan, xb.g_in, xb.glin_in if has_lin else None,
                                     rowmap=None, out=xb.g_rows,
                                     out_lin=xb.g_lin if has_lin else None)
            self._span("scatter", t)
            t = self._mark("adam")
            hip_ops.adam_deferred_rows(self.E_tab, self.m_E, self.v_E, self.w_tab, self.m_w,
                                       self.v_w, self.last, xb.gplan, step_hint,
                                       self.step_table, self.betas, self.eps,
                                       self.weight_decay, grad_rows=xb.g_rows,
                                       grad_lin=xb.g_lin if has_lin else None,
                                       step_dev=self.step_cur)
            self._span("adam", t)
        # 6. the dense gradient (and the loss) over the ranks, then the dense Adam
        t = self._mark("exchange")
        self._join_wgrad()
        if f:  # the dense gradient and, in its tail, the batch loss: one collective
            allreduce_sum_(self._grad_ext, self.group, force=f)
            b.loss.div_(n)
        self._span("exchange", t)
        self._adam_dense(step_hint)
        hip_ops.step_end(self.step_ctr, b.loss, self.loss_sum)
        return b.loss

    def _sharded_fwd_bwd(self, ids, y, b, T, T_lin, bias, mean_div, F):
        """Forward + backward over the compact table T (ids: slot -> unique ordinal), the
        per-row gradient sums into b.grad_rows / b.grad_lin (plan order); returns gz."""
        gv = self.grad_views
        B = ids.shape[0]
        if self.kind == "FM":
            t = self._mark("gather")
            hip_ops.fm_forward(ids, T, T_lin, bias, want_sum=True, labels=y, mean_div=mean_div,
                               want_p=False, out=b.fm)
            self._span("gather", t)
            gz = b.fm.gz
            hip_ops.tensor_sum(gz, out=gv["bias"].view(1))
        else:
            gz = self._deepfm_forward_backward(ids, y, b, T, T_lin, bias, mean_div)
        t = self._mark("scatter")
        xb = getattr(self, "_xb_cur", None)
        if xb is not None and self._grads_to_chunks and not self.keep_grads:
            # the row sums straight into the exchange chunks (no compact sums + pack pass)
            if self.kind == "IPNN":
                hip_ops.shard_row_grads(b.plan, xb.C, xb.offsets, xb.g_out, K=self.K,
                                        vals=b.dslot)
            else:
                hip_ops.shard_row_grads(b.plan, xb.C, xb.offsets, xb.g_out, K=self.K, F=F, emb=T,
                                        gz=gz, sum_e=b.fm.sum_e, dx=b.dx,
                                        lin=T_lin is not None)
        elif self.kind == "IPNN":  # per-slot gradients (through the pair products) summed per row
            hip_ops.segment_sum_rows(b.plan, b.dslot, out=b.grad_rows)
        else:
            hip_ops.fm_embedding_grad(b.plan, F, T, gz, b.fm.sum_e, b.dx, None,
                                      grad_rows=b.grad_rows, grad_lin=b.grad_lin, compact=True)
        self._span("scatter", t)
        if self.kind != "FM":  # the dense-parameter gradients, on the weight-gradient stream
            self._weight_grads(b, gz)
        else:
            hip_ops.tensor_sum(b.fm.loss_elem, scale=1.0 / B, out=b.loss)
        return gz

    # -------------------------------------------------- variable-split (comparison) ------
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

    def _step_varsplit(self, x, y, global_batch=None, next_x=None) -> torch.Tensor:
        """The variable-split protocol: per-owner counts all-to-all (sizes to the host),
        variable all-to-alls of ids, rows and gradients; eager."""
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
        bias = self.views.get("bias")
        has_lin = self.w_tab is not None
        self._sync_weight_planes()
        self._bound_staleness()
        main, ps = hip_ops.current_stream(), self._plan_stream
        xkey = self._xkey(x)
        ahead = [] if next_x is None else (
            [next_x] if isinstance(next_x, torch.Tensor) else list(next_x))
        ahead = [n for n in ahead if n.is_cuda and n.dim() == 2 and n.shape[1] == F
                 and self._xkey(n) != xkey]
        ev_start = torch.cuda.Event()
        ev_start.record(main)
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
                plan.build(self._plan_ids(x), self._V_plan, err_flag=self.err)
                plan.shard_counts(self.shard_rows, ws, out=counts)
        b.plan = plan
        with torch.cuda.stream(ps):
            send_c, recv_c = exchange_counts(counts, self._count_group)
            ev_plan = torch.cuda.Event()
            ev_plan.record(ps)
        main.wait_event(ev_plan)
        self._span("plan", t)
        t = self._mark("exchange")
        req = alltoallv(plan.unique_rows, send_c, recv_c, self.group)
        hip_ops.ids_add_(req, -self.row_lo)
        self._span("exchange", t)
        t = self._mark("catchup")
        hip_ops.adam_deferred_catchup_ids(self.E_tab, self.m_E, self.v_E, self.w_tab, self.m_w,
                                          self.v_w, self.last, req, self.rowmap, self.step_done,
                                          self.step_table, self.step_count + 1, self.betas,
                                          self.eps, self.weight_decay)
        self._span("catchup", t)
        t = self._mark("exchange")
        rows = hip_ops.embedding_gather(self.E_tab, req)
        T = alltoallv(rows, recv_c, send_c, self.group)
        T_lin = None
        if has_lin:
            lin = hip_ops.embedding_gather(self.w_tab.view(-1, 1), req)
            T_lin = alltoallv(lin, recv_c, send_c, self.group).view(-1)
        self._span("exchange", t)
        ids = plan.slot_to_unique(out=self._slot2u)[:B * F].view(B, F)
        self._sharded_fwd_bwd(ids, y, b, T, T_lin, bias, mean_div, F)
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
        b.gplan.build(req, self.E_tab.shape[0])
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
        hip_ops.step_end(self.step_ctr, b.loss, self.loss_sum)
        for n in ahead:  # the next batches' plans and counts, concurrent with this step
            k = self._xkey(n)
            if k in self._pending:
                continue
            ps.wait_event(ev_start)
            n.record_stream(ps)
            with torch.cuda.stream(ps):  # allocated from the plan stream's pool: its writer
                P = self._plan_for(n)
                c = torch.empty(ws, dtype=torch.int64, device=self.device)
                P.build(self._plan_ids(n), self._V_plan, err_flag=self.err)
                P.shard_counts(self.shard_rows, ws, out=c)
                ev = torch.cuda.Event()
                ev.record(ps)
            self._pending[k] = ev
            self._ahead_counts[k] = c
        return b.loss

    # ---------------------------------------------------------------- the tables ------
    def gather_tables(self, device=None) -> tuple[torch.Tensor, torch.Tensor | None]:
        """Full (E [V,K], w [V,1] or None for InnerPNN) assembled from every rank's shard
        (after a flush); every rank calls it. device: where the result goes (default: the
        trainer's device; "cpu" for a table larger than one GPU: the shards then travel one
        at a time, nothing of full size is allocated on a device)."""
        self.flush()
        dev = torch.device(device) if device is not None else self.device
        E_loc = self.E_tab[:self.V_tab]
        w_loc = self.w_tab[:self.V_tab] if self.w_tab is not None else None
        if self.world_size == 1:
            return (E_loc.to(dev, copy=True),
                    w_loc.to(dev, copy=True).view(-1, 1) if w_loc is not None else None)
        gloo = dist.get_backend(self.group) == "gloo"

        def gather(tab, width):
            send = torch.zeros(self.shard_rows, width, dtype=tab.dtype, device=tab.device)
            send[:self.V_tab] = tab.reshape(self.V_tab, width)
            n = self.world_size
            if dev.type == "cuda" and not gloo:
                out = torch.empty(self.shard_rows * n, width, dtype=tab.dtype, device=dev)
                dist.all_gather_into_tensor(out, send, group=self.group)
                if self.layout == "cyclic":  # row q*N + r = shard r's local row q
                    return out.view(n, self.shard_rows, width).transpose(0, 1).reshape(
                        -1, width)[:self.V].contiguous()
                return out[:self.V]
            out = torch.empty(self.V, width, dtype=tab.dtype, device=dev)
            buf = send.cpu() if gloo else torch.empty_like(send)
            for r in range(n):  # one shard in flight at a time
                src = dist.get_global_rank(self.group, r) if self.group is not None else r
                if r == self.rank:
                    buf.copy_(send)
                dist.broadcast(buf, src=src, group=self.group)
                cnt = self._rows_of(r)
                self._cut(out, r).copy_(buf[:cnt])
            return out

        return gather(E_loc, self.K), (gather(w_loc, 1) if w_loc is not None else None)
