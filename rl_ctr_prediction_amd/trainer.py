"""The fused CTR training step — the hot path of this repo.

Replaces the per-batch body of ``all_main/pretrain_main.py:train`` (67-83):
``y = model(x); loss = BCELoss(y, labels); model.zero_grad(); loss.backward();
optimizer.step()`` for FM (p_model.py:28-57) and DeepFM (p_model.py:256-324) with
torch.optim.Adam(lr, weight_decay) — reference semantics, including DENSE Adam (every
embedding row moves every step) and the unfused BCE∘sigmoid gradient.

Per step, on one HIP stream (all kernels from libctr_hip.so):
  FM:      fm_forward(+BCE head) -> sum(gz) -> sparse plan -> per-row grad sums
           -> Adam(E, w) dense pass -> Adam(bias)
  DeepFM:  fm_forward(+flat gather) -> 2 x GEMM(bias+ReLU+dropout) -> head(Linear(200,1)
           + sigmoid + BCE + dH2) -> GEMM dH1 (mask epilogue) -> GEMM dX -> 3 weight-grad
           GEMMs (split-K, deterministic) + column sums -> sparse plan -> per-row grad
           sums (FM + MLP-input grads) -> Adam(E, w) dense pass -> Adam(flat MLP)
The dense [V,K] gradient is never materialised.

Optimizer modes (identical results, bitwise — tests/test_gpu_deferred.py):
  "deferred" (default): deferred-exact dense Adam (temporal blocking, csrc/adam.hip): the
      batch's rows are brought up to date before the forward reads them, updated with their
      gradient after the backward, and every other row replays its missed g = wd*p steps in
      registers at flush() — called automatically before model.forward / state_dict and by
      reset_optimizer(), and by the driver at every epoch end.
  "dense": one streaming pass over all V rows every step (rowmap-gated gradients,
      24 B/element/step).
"""
from __future__ import annotations

import contextlib
import gc
import os
import weakref
from dataclasses import dataclass

import torch
import torch.nn as nn

from . import hip_ops
from ._lib import lib
from .distributed import allgather_sparse_rows, allreduce_sum_, world
from .p_model import FM, DeepFM, InnerPNN


@contextlib.contextmanager
def graph_capture(g, **kw):
    """torch.cuda.graph with Python's cyclic GC paused: a collection during the capture
    could destroy another trainer's captured graphs (HIP calls that are illegal while a
    stream captures -> abort)."""
    gc.collect()  # dead cycles holding captured graphs die here, outside any capture
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(g, **kw):
            yield
    finally:
        if was:
            gc.enable()


def live_pool(owner):
    """The graph memory pool handle of `owner` (a trainer / PolicyGradient) for its next
    capture: torch frees a shared pool once every graph captured into it is gone, and a
    capture into the freed pool's handle trips an allocator assert (and leaves the RNG in
    capture state), so an owner whose step graphs were all dropped starts a new pool."""
    if not owner._graphs:
        owner._graph_pool = torch.cuda.graph_pool_handle()
    return owner._graph_pool


def flush_hooks(model: nn.Module, trainer) -> None:
    """forward / state_dict pre-hooks that flush the trainer's deferred rows, holding the
    trainer weakly (no model <-> trainer cycle: a dropped trainer is freed at once)."""
    ref = weakref.ref(trainer)

    def flush(*_):
        t = ref()
        if t is not None:
            t.flush()

    def drain(*_):  # a pending weight-gradient tail is applied before the loaded values land
        t = ref()
        if t is not None:
            t._drain_tail()
    model.register_forward_pre_hook(flush)
    model.register_state_dict_pre_hook(flush)
    model._register_load_state_dict_pre_hook(drain)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

DEEPFM_DENSE = ("bias", "mlp.0.weight", "mlp.0.bias", "mlp.3.weight", "mlp.3.bias",
                "mlp.6.weight", "mlp.6.bias")
FM_DENSE = ("bias",)
IPNN_DENSE = DEEPFM_DENSE[1:]  # InnerPNN: the MLP only (no linear term, no bias)
_MLP_KINDS = ("DeepFM", "IPNN")


class InputSlot:
    """Fixed device buffers one batch is copied into before its step: the ids [B,F] (the
    caller's dtype), the labels [B] as float32 and the batch's sparse plan. The step graph
    of a slot is captured once against these addresses and replayed for every batch that
    passes through the slot, so a stream of fresh batches replays the same graphs (the
    reference trains on a new batch every iteration, all_main/pretrain_main.py:71-78)."""

    __slots__ = ("shape", "index", "ids", "y", "y_key", "plan", "ev", "plan_graph",
                 "done_ev", "stream_i", "stage_stream", "cap", "counts", "slot2u", "gen",
                 "planned")

    def __init__(self, shape, index: int, device):
        B, F, dtype = shape
        self.shape, self.index = shape, index
        self.ids = torch.empty(B, F, dtype=dtype, device=device)
        self.y = torch.empty(B, dtype=torch.float32, device=device)
        self.y_key = None       # staged ahead with the labels too: the labels tensor's key
        self.plan = hip_ops.SparsePlanBuffers(B * F, device)
        self.ev = None          # staged ahead: the copy + plan on the plan stream recorded here
        self.plan_graph = None  # the plan build of this slot, captured on its plan stream
        self.done_ev = None     # the slot's staging event (one per slot, re-recorded)
        self.stream_i = 0
        self.stage_stream = None  # the plan stream its last staging ran on
        self.cap = self.counts = None  # ShardedCTRTrainer: per-owner runs of the plan
        self.slot2u = None  # ShardedCTRTrainer: slot -> unique ordinal, built with the plan
        self.gen = 0  # ShardedCTRTrainer: staging generation (which contents the plan measured)
        self.planned = True  # False: staged ids copied, plan not built yet (plan_in_graph)


@dataclass
class _Bufs:
    B: int
    fm: hip_ops.FMForward
    plan: hip_ops.SparsePlanBuffers    # the plan of the step's batch
    grad_rows: torch.Tensor
    grad_lin: torch.Tensor
    h1: torch.Tensor | None = None
    h2: torch.Tensor | None = None
    head: dict | None = None
    dx: torch.Tensor | None = None
    # exact three-plane bf16 splits (hip_ops.Planes) of the MLP GEMM operands, written by
    # their producers; the GEMMs read them in the stored orientation (csrc/gemm_planes.hip)
    xp: hip_ops.Planes | None = None    # MLP input X [B, W]
    h1p: hip_ops.Planes | None = None   # H1 [B, H1]
    dh2p: hip_ops.Planes | None = None  # dH2 [B, H2]
    dh1p: hip_ops.Planes | None = None  # dH1 [B, H1]
    loss: torch.Tensor | None = None
    gplan: hip_ops.SparsePlanBuffers | None = None
    g_rows: torch.Tensor | None = None
    g_lin: torch.Tensor | None = None
    dslot: torch.Tensor | None = None  # IPNN: per-slot embedding gradients [S, K]
    zero: torch.Tensor | None = None   # IPNN: the (absent) FM logit, zeros [B]
    plan_own: hip_ops.SparsePlanBuffers | None = None  # the shape's plan without lookahead
    xps: dict | None = None  # pipelined tail: X plane buffers by index (_xp_for)
    xp_idx: int = 0


class FusedCTRTrainer:
    """Fused forward + BCE + backward + dense Adam for FM / DeepFM.

    Args mirror ``torch.optim.Adam(model.parameters(), lr, betas, eps, weight_decay)``.
    The model's dense parameters (FM bias, DeepFM MLP) are re-pointed into one flat
    buffer (same Parameter objects, same state_dict), so the dense Adam and the
    data-parallel all-reduce are one launch each.
    """

    def __init__(self, model: nn.Module, lr: float = 1e-3, weight_decay: float = 0.0,
                 betas=(0.9, 0.999), eps: float = 1e-8, process_group=None, seed: int | None = None,
                 optimizer_mode: str = "deferred"):
        if not isinstance(model, (FM, DeepFM, InnerPNN)):
            raise TypeError("FusedCTRTrainer drives FM, DeepFM or InnerPNN")
        self.model = model
        self.kind = ("DeepFM" if isinstance(model, DeepFM) else
                     "IPNN" if isinstance(model, InnerPNN) else "FM")
        self.lr, self.weight_decay, self.betas, self.eps = float(lr), float(weight_decay), betas, eps
        self.group = process_group
        E = model.feature_embedding.weight
        self.device = E.device
        if self.device.type != "cuda":
            raise RuntimeError("FusedCTRTrainer needs the model on a ROCm device")
        self.V, self.K = self._vocab_size(E), E.shape[1]
        named = dict(model.named_parameters())
        self.dense_names = {"DeepFM": DEEPFM_DENSE, "FM": FM_DENSE, "IPNN": IPNN_DENSE}[self.kind]
        # 16-B aligned views (offsets multiples of 4 floats): the GEMMs read the weights
        # through the float4 / LDS-DMA path only when a row start is 16-B aligned
        self.offsets, total = {}, 0
        for n in self.dense_names:
            self.offsets[n] = total
            total += (named[n].numel() + 3) // 4 * 4
        flat = torch.zeros(total, dtype=torch.float32, device=self.device)
        # the dense gradient with 4 floats of tail room: the row-sharded step all-reduces the
        # batch loss there, in the gradient's own collective (sharded.py)
        self._grad_ext = torch.zeros(total + 4, dtype=torch.float32, device=self.device)
        self.flat_grad = self._grad_ext[:total]
        self.views, self.grad_views = {}, {}
        for n in self.dense_names:
            p, off = named[n], self.offsets[n]
            k = p.numel()
            flat[off:off + k].copy_(p.data.reshape(-1))
            p.data = flat[off:off + k].view_as(p)
            self.views[n] = p.data
            self.grad_views[n] = self.flat_grad[off:off + k].view_as(p)
        self.flat = flat
        self.m_flat = torch.zeros_like(flat)
        self.v_flat = torch.zeros_like(flat)
        # the embedding rows this trainer's optimiser owns: all of them here, one shard in
        # ShardedCTRTrainer (rl_ctr_prediction_amd/sharded.py)
        self.row_lo, self.row_hi = self._table_rows()
        self.V_tab = self.row_hi - self.row_lo
        self.E_tab = self._own_rows(E.data)
        n_rows = self.E_tab.shape[0]  # V_tab (+ a spare row under row sharding)
        self.m_E = torch.zeros_like(self.E_tab)
        self.v_E = torch.zeros_like(self.E_tab)
        if self.kind == "IPNN":  # no linear table: every lin pointer of the ABI is NULL
            self.w_tab = self.m_w = self.v_w = None
        else:
            self.w_tab = self._own_rows(model.linear.weight.data)
            self.m_w = torch.zeros(n_rows, dtype=torch.float32, device=self.device)
            self.v_w = torch.zeros_like(self.m_w)
        if optimizer_mode not in ("deferred", "dense"):
            raise ValueError(f"optimizer_mode must be 'deferred' or 'dense', not {optimizer_mode!r}")
        self.deferred = optimizer_mode == "deferred"
        # dense mode: row -> compact gradient slot map; deferred mode: the owner scratch of
        # the plan-free catch-up (csrc/adam.hip deferred_mark_kernel)
        self.rowmap = torch.full((n_rows,), -1, dtype=torch.int32, device=self.device)
        self.last = torch.zeros(n_rows, dtype=torch.int32, device=self.device)
        # device step counters: [0] completed steps, [1] the step in flight (ctr_step_begin/end)
        # initialised to {0, 1}: ctr_step_end advances both, so no step-begin launch is needed
        self.step_ctr = torch.tensor([0, 1], dtype=torch.int32, device=self.device)
        self.step_done, self.step_cur = self.step_ctr[0:1], self.step_ctr[1:2]
        # fused scatter + Adam apply (one process, deferred mode); keep_grads keeps every
        # row's gradient sum in b.grad_rows / b.grad_lin (tests read them)
        self.fuse_apply = os.environ.get("CTR_FUSE_APPLY", "1") != "0"
        # smallest K the fused apply is used at (A/B: CTR_FUSE_APPLY_MIN_K)
        self.fuse_apply_min_k = int(os.environ.get("CTR_FUSE_APPLY_MIN_K", "16"))
        # capture order of the step's first fork: the plan first where it is the critical
        # path (FM: the forward / backward are short; C2 31.6 vs 28.4 M ex/s), the catch-up
        # and forward first where they are (MLP kinds; C3 12.39 vs 11.67 M ex/s)
        env = os.environ.get("CTR_PLAN_FIRST")
        self.plan_first = (env == "1") if env in ("0", "1") else self.kind == "FM"
        self.keep_grads = False
        # input staging (single process): every batch is copied into a fixed slot of its
        # shape (InputSlot) and the step graph of that slot is replayed, so fresh batches
        # never miss the graph cache. Plan lookahead (step(..., next_x=)): the next batches
        # are copied into slots of their own on a plan stream and their sparse plans built
        # there (each slot's plan build is its own small graph), concurrently with this step;
        # the step that trains on one of them waits for it before it starts. A ring of
        # lookahead + 1 slots per shape: a slot is restaged only after the step that used it
        # (the plan stream waits for everything enqueued before the current step)
        self._rings: dict = {}     # (B, F, dtype) -> [InputSlot]
        self._staged: dict = {}    # ids key of a batch staged ahead -> its InputSlot
        self.max_slots = 8
        self.captures = 0          # step graphs captured (tests: bounded, batch-independent)
        self._ev_start = None
        # lookahead (every kind): the next batches' ids are staged and planned on the plan
        # stream, so the step graph starts with no copy and no plan branch, and catches its
        # rows up over the plan's unique rows in one launch. FM: C2 35.5 -> 50.9 M ex/s; C3
        # streaming fresh batches 11.94 -> 12.48 M ex/s (two alternating runs each; with
        # cycled batches it had measured 12.7 vs 12.8, the in-step copies then absent)
        env = os.environ.get("CTR_PLAN_LOOKAHEAD")
        self.plan_lookahead = (env == "1") if env in ("0", "1") else True
        # bounded staleness of deferred Adam: every `flush_every` steps all rows are brought
        # to the current step (one tiled flush pass), so a row a batch touches has missed at
        # most that many steps and the in-step catch-up replays stay short under a stream
        # of fresh batches (0: only at forward / state_dict / epoch end)
        self.flush_every = int(os.environ.get("CTR_FLUSH_EVERY", "32"))
        self._flushed_at = 0
        self._vec_ok = self.K % 4 == 0 and 64 % (self.K // 4 or 1) == 0 and self.K <= 256
        # every stream of this trainer has a HIP handle of its own (_new_stream): the scratch
        # buffers of hip_ops.Workspace are per stream handle, and torch hands streams out of
        # a 32-stream pool round-robin, so two roles could otherwise alias one stream and
        # share scratch while running concurrently (the step graphs are captured on the
        # trainer's own capture stream for the same reason, not on torch's global one)
        self._own_streams: list = []
        # scratch owned by this trainer alone: its captured graphs reference no buffer that
        # another object's launches use (hip_ops.Workspace)
        self._scratch = hip_ops.Workspace()
        self._capture_stream = self._new_stream()
        self._side = self._new_stream() if self.deferred and self._vec_ok else None
        # the weight-gradient work shares the plan's side stream (it starts after the head,
        # long after the plan is built): the captured graph then has exactly two parallel
        # lists — the critical path and one side list — and the HIP graph executor cannot
        # map two independent side lists onto one hardware queue in the wrong order (seen
        # with three: the plan queued behind the weight gradients, +100 us per step)
        self._wgrad_stream = None
        if self.kind in _MLP_KINDS:
            self._wgrad_stream = self._side if self._side is not None else self._new_stream()
            # experiment: the weight-gradient stream on a fraction of the
            # CUs, so dW0 leaves the rest to the scatter beside it. The mask holds for eager
            # launches only — a graph branch forked onto a masked stream runs on every CU
            # (tools/cumask_probe.hip) — so it was measured with graphs off: C3 5.2-5.8 vs
            # 13.1-13.3 M ex/s unmasked, the masked queue's kernels no longer overlapping the
            # main queue's (profiles/r06_cumask.txt). Not a default.
            frac = os.environ.get("CTR_WGRAD_CU_FRAC")
            if frac:
                n_cus = torch.cuda.get_device_properties(self.device).multi_processor_count
                self._wgrad_stream = hip_ops.cu_masked_stream(
                    hip_ops.cu_mask_words(n_cus, float(frac)), device=self.device)
        # the MLP weights' planes: rewritten by the dense Adam with every update
        # (ctr_adam_dense_planes), re-split from the fp32 parameters (the source of truth:
        # state_dict / load_state_dict see fp32) whenever those changed outside the trainer
        self._wplanes = None
        self._wver = None
        if self.kind in _MLP_KINDS:
            w0, w1 = self.views["mlp.0.weight"], self.views["mlp.3.weight"]
            self._wplanes = (hip_ops.Planes(*w0.shape, self.device),
                             hip_ops.Planes(*w1.shape, self.device))
        # created on first use: every HIP stream takes one of the process's few hardware
        # queues (GPU_MAX_HW_QUEUES = 4), and streams beyond that share queues in order
        self._plan_stream = None
        if self._side is not None:
            self._plan_stream = self._new_plan_stream()
        # lookahead plans may alternate over n_plan_streams streams (each key keeps its own:
        # its captured graph holds that stream's scratch), two plans in flight at once.
        # Default 2: with the host off the step's critical path (step(): 30 us of Python),
        # C2 two streams 50.5 / 54.8 / 53.4 vs one 50.5 / 48.9 / 47.3 M ex/s (alternating
        # runs, tools/c2_knobs3.sh); while the host paced the step one stream measured faster
        self.n_plan_streams = int(os.environ.get("CTR_PLAN_STREAMS", "2"))
        # a staged batch's copy + plan alternate over the plan streams in staging order, so
        # two consecutive plans never queue on one stream (with a ring of three slots, a
        # slot-index rule put slots 0 and 2 on one stream: their plans ran back to back, two
        # in one step and none in the next)
        self._stage_seq = 0
        self._extra_plan_streams: list = []
        # where a lookahead plan starts: after everything enqueued before the step that
        # stages it (False), or after that whole step (True). Traced at C3 (round 5, kernel
        # trace of the timed region): a plan that starts with the step lands beside the
        # backward's weight-gradient GEMMs on every other step (its 26 column-sort blocks hold
        # 26 CUs for ~125 us, dW0's one-block-per-CU grid then runs a second wave: 84 -> 132
        # us, the step 410 -> 462 us); started after the step it runs beside the next step's
        # catch-up and gather (HBM- and latency-bound, no slowdown measured) and is ready a
        # whole step before it is needed. CTR_PLAN_AFTER_STEP=0/1 overrides the default
        # (on for the MLP kinds, whose steps are long against the plan; FM steps at C2 are
        # about the plan's length)
        env = os.environ.get("CTR_PLAN_AFTER_STEP")
        self.plan_after_step = (env == "1") if env in ("0", "1") else False
        self._ev_end = None
        # opt-in (CTR_PLAN_IN_GRAPH=1): the next batch's plan inside this step's
        # graph, on the side list between dW1 and the dX join; a staged batch is then only
        # copied ahead. Traced at C3 (round 6, profiles/r06_c3_timelines.txt): a plan built on
        # a plan stream lands wherever its queue lets it — beside dX (free), beside dW0 on some
        # steps (+50 us), beside the next catch-up / gather on others — so the steps' walls
        # spread 394-460 us. In the side list the column sort stretches to ~83 us beside dX
        # and delays dW0 until after the scatter: every step 435-450 us (scatter 40 us alone
        # instead of 84 beside dW0, dW0 66 alone instead of 85, but serial), C3 12.73 / 12.78
        # / 12.92 vs 13.32 / 13.32 / 13.39 M ex/s off (alternating): off by default. FM (the
        # plan on the side list beside the gather and scatter, joined before the tail: one
        # graph launch per step instead of two) at C2: 37.9 / 40.0 / 47.7 / 39.8 vs 49.3 /
        # 55.4 / 49.2 / 55.7 M ex/s off — the join costs the GPU more than the launch saves
        env = os.environ.get("CTR_PLAN_IN_GRAPH")
        self.plan_in_graph = (env == "1") and self.kind in _MLP_KINDS + ("FM",)
        self._next_plan = None  # the staged slot whose plan the step being launched builds
        # cross-step pipelining of the MLP kinds' weight-gradient tail (one process, deferred
        # mode): the largest weight gradient dW0 = dH1^T X and the MLP weights' Adam of step t
        # run at the START of step t+1's graph, on the side stream beside its catch-up and
        # gather (which read no MLP weight), joined before its first GEMM — instead of beside
        # step t's scatter chain, where the two shared the CUs and HBM. The
        # MLP input planes X are per input slot (step t+1's gather writes its slot's
        # while dW0 of step t reads step t's slot's; _pipe_state). A pending tail is applied by flush() (model
        # forward / state_dict / load_state_dict hooks, the epoch end) and by _drain_tail().
        # Opt-in (CTR_PIPELINE_WGRAD=1): bitwise the in-step tail, but measured slower at C3
        # (11.77 / 11.89 vs 12.77 / 12.62 M ex/s, alternating): the scatter chain loses dW0's
        # contention (105 -> 76 us) but the gather beside dW0 takes 85 us instead of 28
        # (profiles/r05_pipelined_tail.txt)
        env = os.environ.get("CTR_PIPELINE_WGRAD")
        self._pipe = (self.kind in _MLP_KINDS and self.deferred and self._side is not None
                      and world()[1] == 1 and env == "1")
        # (bufset, X planes, their index) of the step whose dW0 + MLP Adam is pending
        self._tail = None
        self.step_table = hip_ops.AdamStepTable(self.lr, self.betas, self.device)
        self._dirty = False
        if self.deferred:  # nothing may read a table with rows still owed steps
            flush_hooks(model, self)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        # every step's mean loss added in float64 by its last launch (the driver's epoch sum)
        self.loss_sum = torch.zeros(1, dtype=torch.float64, device=self.device)
        self.step_count = 0
        self._bufs: _Bufs | None = None
        self._bufsets: dict = {}
        self.seed = int(torch.initial_seed() if seed is None else seed) & (2**63 - 1)
        # HIP-graph replay of the single-process step (see step()): per shape at most
        # 2 x ring-size graphs (slot x plan-built-ahead), independent of the batch count
        self.use_graphs = True
        self.max_graphs = 24
        self._graphs: dict = {}
        self._graph_pool = torch.cuda.graph_pool_handle()
        self._graph_tab_version = self.step_table.version
        # bench hook: {"adam": [], "gather": [], ...} -> [(start, end, work)] HIP events
        # recorded on the launch stream around those kernels; only the keys present in the
        # dict are instrumented (each event is a queue packet: keep the timed region lean)
        self.timing: dict | None = None

    def __del__(self):
        # a captured graph must not be destroyed while it still runs: plan-stream replays
        # (lookahead) are not ordered before anything the caller synchronises with
        try:
            if getattr(self, "_graphs", None) or getattr(self, "_rings", None):
                torch.cuda.synchronize(self.device)
        except Exception:  # interpreter shutdown
            pass

    def _table_rows(self) -> tuple[int, int]:
        return 0, self.V

    def _vocab_size(self, E) -> int:
        return E.shape[0]

    def _own_rows(self, t: torch.Tensor) -> torch.Tensor:
        """This trainer's rows of a table Parameter's data (ShardedCTRTrainer: the data IS
        the shard)."""
        return t[self.row_lo:self.row_hi]

    def _mark(self, key):
        if self.timing is None or key not in self.timing:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def _span(self, key, start, work=None):
        if start is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.timing[key].append((start, ev, work))

    def _gemm(self, *args, **kw):
        """hip_ops.gemm with a timing span carrying the product's flop count."""
        t = self._mark("gemm")
        out = hip_ops.gemm(*args, **kw)
        if t is not None:
            a, bb = args[0], args[1]
            ta, tb = kw.get("trans_a", False), kw.get("trans_b", False)
            M, K = (a.shape[1], a.shape[0]) if ta else a.shape
            N = bb.shape[0] if tb else bb.shape[1]
            self._span("gemm", t, 2.0 * M * N * K)
        return out

    def _gemm_planes(self, a, b, a_rc, b_rc, M, N, K, **kw):
        """hip_ops.gemm_planes with a timing span carrying the product's flop count."""
        t = self._mark("gemm")
        out = hip_ops.gemm_planes(a, b, a_rc, b_rc, **kw)
        self._span("gemm", t, 2.0 * M * N * K)
        return out

    def _linear(self, x, w, b, **kw):
        t = self._mark("gemm")
        out = hip_ops.linear(x, w, b, **kw)
        if t is not None:
            self._span("gemm", t, 2.0 * x.shape[0] * w.shape[0] * x.shape[1])
        return out

    # ----------------------------------------------------------------- optimiser -----
    def flush(self) -> None:
        """Apply the pending weight-gradient tail (pipelined MLP kinds) and bring every
        embedding row up to the last completed step (deferred mode): every parameter and
        moment is then the reference's after the last step. The plan streams only read
        staged ids and write plans: nothing to wait for."""
        self._drain_tail()
        self._flush_table()

    def _flush_table(self) -> None:
        """The embedding rows up to the last completed step (deferred mode)."""
        self._flushed_at = self.step_count
        if self.deferred and self._dirty and self.step_count > 0:
            t = self._mark("flush")
            hip_ops.adam_deferred_flush(self.E_tab, self.m_E, self.v_E,
                                        self.w_tab, self.m_w, self.v_w, self.last,
                                        self.step_count, self.step_table, self.betas, self.eps,
                                        self.weight_decay)
            self._span("flush", t)
        self._dirty = False

    def reset_optimizer(self, lr: float | None = None) -> None:
        """What ``torch.optim.Adam(...)`` re-created every epoch does
        (all_main/pretrain_main.py:153): fresh moments, step 0 — with `lr`, at a new
        learning rate (main/pretrain_main.py:180-181: ``learning_rate += 1e-4`` then a new
        Adam): the per-step scalars are rewritten in place (captured graphs stay valid)."""
        self.flush()
        if lr is not None:
            self.lr = float(lr)
            self.step_table.set_lr(self.lr)
        for t in (self.m_flat, self.v_flat, self.m_E, self.v_E, self.m_w, self.v_w):
            if t is not None:
                t.zero_()
        self.last.zero_()
        self.step_ctr.copy_(torch.tensor([0, 1], dtype=torch.int32))
        self.step_count = 0
        self._flushed_at = 0

    def _bound_staleness(self) -> None:
        """Flush once `flush_every` steps have passed since the last flush: no row is then
        more than that many steps behind when a batch reads it."""
        if (self.deferred and self.flush_every > 0
                and self.step_count - self._flushed_at >= self.flush_every):
            self._flush_table()  # the tables only: the pipelined tail stays pending

    def optimizer_state_dict(self) -> dict:
        """torch.optim.Adam-compatible state_dict (parameter order = model.parameters())."""
        self.flush()
        named = list(self.model.named_parameters())
        m = {n: v for n, v in zip(self.dense_names, self._split(self.m_flat))}
        v = {n: v for n, v in zip(self.dense_names, self._split(self.v_flat))}
        m["feature_embedding.weight"], v["feature_embedding.weight"] = self.m_E, self.v_E
        if self.m_w is not None:
            m["linear.weight"], v["linear.weight"] = self.m_w.view(-1, 1), self.v_w.view(-1, 1)
        state = {i: {"step": torch.tensor(float(self.step_count)), "exp_avg": m[n].clone(),
                     "exp_avg_sq": v[n].clone()} for i, (n, _) in enumerate(named)}
        return {"state": state if self.step_count else {},
                "param_groups": [{"lr": self.lr, "betas": self.betas, "eps": self.eps,
                                  "weight_decay": self.weight_decay, "amsgrad": False,
                                  "params": list(range(len(named)))}]}

    def _split(self, flat):
        out = []
        for n in self.dense_names:
            k, off = self.views[n].numel(), self.offsets[n]
            out.append(flat[off:off + k].view_as(self.views[n]))
        return out

    # --------------------------------------------------------------------- buffers ---
    def _buffers(self, B: int, F: int) -> _Bufs:
        # one buffer set per batch shape, never freed: captured HIP graphs hold their
        # addresses (a ragged last batch must not invalidate the full-batch graphs)
        b = self._bufsets.get((B, F))
        if b is not None:
            self._bufs = b
            return b
        dev, K = self.device, self.K
        e = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        deep = self.kind in _MLP_KINDS
        W = F * K + (F * (F - 1) // 2 if self.kind == "IPNN" else 0)  # MLP input width
        # DeepFM writes its MLP input straight as planes (b.xp): no fp32 copy of X
        x_fp32 = deep and not (self.kind == "IPNN" or hip_ops.fm_forward_planes_ok(K, F))
        fm = hip_ops.FMForward(z=e(B), sum_e=e(B, K), emb_out=e(B, W) if x_fp32 else None,
                               p=None, loss_elem=e(B), gz=e(B))
        S = B * F
        b = _Bufs(B=B, fm=fm, plan=hip_ops.SparsePlanBuffers(S, dev), grad_rows=e(S, K),
                  grad_lin=e(S), loss=e(1))
        b.plan_own = b.plan
        if deep:
            mlp = self.model.mlp
            H1, H2 = mlp[0].out_features, mlp[3].out_features
            b.h1, b.h2, b.dx = e(B, H1), e(B, H2), e(B, W)
            P = hip_ops.Planes
            # H1 carries a ones column in its padding: dW1 then returns the bias gradient
            # db1 = colsum dH2 as one more output column
            # ... and so does the MLP input X (db0 = colsum dH1 from dW0, CTR_WGRAD_ORDER)
            b.xp = P(B, W, dev, ones_col=True)
            # pipelined tail: one X plane buffer per input slot (+ a spare), _xp_for
            b.xps = {0: b.xp} if self._pipe else None
            b.h1p = P(B, H1, dev, ones_col=True)
            b.dh2p, b.dh1p = P(B, H2, dev), P(B, H1, dev)
            if self.kind == "IPNN":
                b.dslot = e(S, K)
                b.zero = torch.zeros(B, dtype=torch.float32, device=dev)
            # dH2 goes to the GEMMs as planes only: no fp32 copy (6.5 MB a step at C3)
            b.head = dict(z=e(B), p=e(B), loss_elem=fm.loss_elem, gz=fm.gz, dh_pre=None)
        rank, ws = world()
        if ws > 1:
            b.gplan = hip_ops.SparsePlanBuffers(S * ws, dev)
            b.g_rows, b.g_lin = e(S * ws, K), e(S * ws)
        self._bufsets[(B, F)] = b
        self._bufs = b
        return b

    # ------------------------------------------------------------------------ step ----
    def step(self, x: torch.Tensor, y: torch.Tensor, global_batch: int | None = None,
             next_x=None, return_loss: bool = True, next_y=None) -> torch.Tensor | None:
        """One training step on batch (x [B,F] int64/int32, y [B] 0/1). Returns the
        batch's mean BCE as a fresh 1-element device tensor (no host sync), or None with
        return_loss=False (no copy launch; the loss still goes into ``loss_sum``).

        Single process: x and y are copied into a fixed input slot of their shape
        (InputSlot; one D2D copy of the ids and labels) and the slot's step graph — the
        step's ~40 launches captured once, every per-step scalar (the Adam step, the
        dropout stream) read from the device step counter — is replayed, so every fresh
        batch replays the same graph; the first step through a slot runs eagerly and
        captures. x may also be a host tensor (the copy is then the H2D transfer).

        next_x (optional): the ids of the batch(es) the next step(s) will train on — one
        tensor, or a sequence in step order. They are copied into slots of their own and
        their sparse plans (a pure function of the ids) built on a plan stream
        concurrently with this step (single process, deferred mode, plan lookahead on);
        the step that trains on one of them uses that plan instead of building its own on
        its critical path. Two batches ahead hides the plan entirely: its completion is
        then long past when the step waits for it (a cross-queue wait that is still
        pending costs ~15 us). next_x is read on the plan stream after everything enqueued
        before this call: its contents must stay valid until this call's work has run; a
        step with other ids builds its plan as usual. next_y (optional, aligned with next_x):
        those batches' labels, copied into their slots on the plan stream as well, so the
        step that trains on them skips its label copy (the same tensor must then be passed
        as that step's y; any other y is copied as usual). A staged batch is recognised by
        its tensor (address, shape, strides), not its contents: the ids and labels are those
        the tensors held when they were staged, so a tensor refilled in place between its
        staging and its step trains on the staged contents — refill a different buffer.

        Every step also adds its loss (fp64) to the device accumulator ``loss_sum`` inside
        the step's last launch — the driver's epoch loss without a host sync per step
        (read_loss_sum / reset_loss_sum)."""
        with self._scratch.scope():  # this trainer's own scratch (hip_ops.Workspace)
            loss = self._step(x, y, global_batch, next_x, next_y)
            return loss.clone() if return_loss else None

    def reset_loss_sum(self) -> None:
        """Zero the device loss accumulator (on the current stream, in step order)."""
        self.loss_sum.zero_()

    def read_loss_sum(self) -> float:
        """The sum of every step's mean loss since reset_loss_sum(), accumulated on the
        device in float64 in step order: bitwise the reference's per-step
        ``total_loss += loss.item()`` (all_main/pretrain_main.py:79). Syncs once."""
        return float(self.loss_sum.item())

    def _step(self, x: torch.Tensor, y: torch.Tensor, global_batch: int | None = None,
              next_x=None, next_y=None) -> torch.Tensor:
        """step() without the copy of the loss: returns the persistent loss buffer of the
        batch shape (the captured graph writes it in place)."""
        B, F = x.shape
        rank, ws = world()
        mean_div = float(global_batch if global_batch is not None else B * ws)
        self._sync_weight_planes()
        self._bound_staleness()
        if ws != 1:  # replicated data parallel: eager (the exchange sizes live on the host)
            self.step_table.ensure(self.step_count + 1)
            loss = self._launch(x, y, mean_div)
            self._after_step()
            return loss
        # the host side of a step paces small batches (C2: ~70 us of Python per step against
        # ~75 us on the GPU), so each ids tensor's key is computed once and the current
        # stream is looked up once (torch.cuda.current_stream() costs ~4 us)
        shape = (B, F, x.dtype)
        xkey = self._xkey(x)
        nk = []
        ny = {}  # staged labels by ids key
        if next_x is not None and self.plan_lookahead and self._plan_stream is not None:
            xs_ = [next_x] if isinstance(next_x, torch.Tensor) else list(next_x)
            ys_ = ([next_y] if isinstance(next_y, torch.Tensor) else list(next_y)
                   ) if next_y is not None else []
            for j, n in enumerate(xs_):
                k = self._xkey(n)
                if k[1:3] == xkey[1:3] and k != xkey and all(k != kk for _, kk in nk):
                    nk.append((n, k))
                    if j < len(ys_) and ys_[j] is not None and ys_[j].numel() == n.shape[0]:
                        ny[k] = ys_[j]
        main = hip_ops.current_stream()
        slot = self._staged.pop(xkey, None)
        if self._staged:  # staged for batches that did not come next: free their slots
            keep = {k for _, k in nk}
            for k in [k for k in self._staged if k not in keep]:
                ev = self._staged.pop(k).ev
                if ev is not None:  # None: planned in a step graph (main's order)
                    main.wait_event(ev)  # its plan-stream writes come first
        todo = [(n, k) for n, k in nk if k not in self._staged]
        have = slot is not None
        ev_start = None
        if todo:  # everything enqueued before this step (the last users of the slots)
            ev_start = self._start_event()
            ev_start.record(main)
        # the next batch's plan in this step's graph (MLP kinds): its slot is only copied ahead
        pig = (self.plan_in_graph and not self._pipe and self._side is not None
               and self.deferred)
        if have:  # copied (and planned) ahead
            if slot.ev is not None:
                main.wait_event(slot.ev)
                slot.ev = None
            if not slot.planned:  # copied ahead, no step planned it: build it here, first
                self._plan_staged_now(slot, main)
        else:
            slot = self._acquire_slot(shape)
            slot.ids.copy_(x, non_blocking=True)
        if not (have and slot.y_key is not None and slot.y_key == self._xkey(y)):
            slot.y.copy_(y.reshape(-1), non_blocking=True)
        slot.y_key = None
        nxt = None
        if pig and nk:
            n1, k1 = nk[0]
            if k1 not in self._staged:  # stage (copy) it now: this step plans it
                self._stage_ahead(n1, k1, shape, slot, ev_start, main, ny.get(k1), plan=False)
                todo = [(n, k) for n, k in todo if k != k1]
            nxt = self._staged[k1]
            if nxt.planned:
                nxt = None
            elif nxt.ev is not None:
                main.wait_event(nxt.ev)  # its ids copy
                nxt.ev = None
        self._next_plan = nxt
        try:
            if self.use_graphs and self.timing is None:
                loss = self._graph_step(slot, mean_div, have)
            else:
                self.step_table.ensure(self.step_count + 1)
                loss = self._launch(slot.ids, slot.y, mean_div, have, plan=slot.plan,
                                    pipe=self._pipe_state(slot))
                self._after_step()
        finally:
            self._next_plan = None
        if nxt is not None:  # complete in main's order, after this step
            nxt.planned = True
        if todo and self.plan_after_step:  # the staged plans start after this whole step
            if self._ev_end is None:
                self._ev_end = torch.cuda.Event()
            self._ev_end.record(main)
            ev_start = self._ev_end
        for n, k in todo:
            self._stage_ahead(n, k, shape, slot, ev_start, main, ny.get(k), plan=not pig)
        return loss

    def _plan_staged_now(self, s: InputSlot, main) -> None:
        """The plan of a slot staged (copied) ahead that no step graph planned, on its
        staging stream (after its copy), replayed from its own plan graph once captured; the
        main stream waits for it."""
        ps = s.stage_stream if s.stage_stream is not None else self._plan_stream
        torch.cuda.set_stream(ps)
        try:
            self._plan_build_slot(s, ps)
            ev = self._slot_event(s)
            ev.record(ps)
        finally:
            torch.cuda.set_stream(main)
        main.wait_event(ev)
        s.planned = True

    def _plan_build_slot(self, s: InputSlot, ps) -> None:
        """On the current stream ps: slot s's plan (its own captured plan graph once it
        exists)."""
        t = self._mark("plan")
        if s.plan_graph is not None and self.timing is None:
            s.plan_graph.replay()
        else:
            s.plan.build(s.ids, self.V)
            if self.use_graphs and self.timing is None:
                g = torch.cuda.CUDAGraph()
                with graph_capture(g, pool=live_pool(self), stream=ps):
                    s.plan.build(s.ids, self.V)  # captured, not executed
                s.plan_graph = g
        self._span("plan", t)

    def _ring(self, shape) -> list:
        r = self._rings.get(shape)
        if r is None:
            r = self._rings[shape] = []
        return r

    def _new_stream(self):
        """A torch stream whose HIP handle no other stream of this trainer (nor the stream
        current at construction, where the steps are usually issued) has."""
        taken = {s.cuda_stream for s in self._own_streams}
        taken |= {0, torch.cuda.current_stream(self.device).cuda_stream}
        for _ in range(64):
            st = torch.cuda.Stream(device=self.device)
            if st.cuda_stream not in taken:
                self._own_streams.append(st)
                return st
        raise RuntimeError("FusedCTRTrainer: no free stream in torch's stream pool")

    def _new_plan_stream(self):
        """A plan stream (a torch stream of its own, _new_stream). Measured and not kept: plan
        streams at the HIP runtime's low priority (hipStreamCreateWithPriority 1, own queues
        in the low-priority pool): C3 8.7 / 8.7 / 9.3 vs 13.2 / 13.1 / 13.1 M ex/s, C2 48.9 /
        47.1 / 53.2 vs 46.6 / 56.6 / 45.1 — behind a queue of step kernels the plans built
        ahead starve and the steps wait for them."""
        return self._new_stream()

    def _slot_stream(self, stream_i: int):
        """Plan stream number stream_i (created on first use)."""
        while stream_i > len(self._extra_plan_streams):
            self._extra_plan_streams.append(self._new_plan_stream())
        return self._plan_stream if stream_i == 0 else self._extra_plan_streams[stream_i - 1]

    def _acquire_slot(self, shape, exclude=None, ahead: bool = False) -> InputSlot:
        """The lowest-index slot of the shape's ring that no staged batch holds (and that is
        not `exclude`, the current step's); the ring grows up to max_slots. Lowest index
        first keeps the set of (slot, planned-ahead) graphs small: the first step of an
        epoch always lands in slot 0. ahead: the new slot's first writer is its plan stream,
        so its buffers come from that stream's pool (a block the current stream freed during
        this step may still be read by work the plan stream does not wait for)."""
        ring = self._ring(shape)
        busy = {id(s) for s in self._staged.values()}
        if exclude is not None:
            busy.add(id(exclude))
        for s in ring:
            if id(s) not in busy:
                return s
        if len(ring) >= self.max_slots:
            raise RuntimeError(f"FusedCTRTrainer: more than {self.max_slots} batches staged ahead")
        index = len(ring)
        stream_i = index % max(1, self.n_plan_streams)
        if ahead and self._plan_stream is not None:
            with torch.cuda.stream(self._slot_stream(stream_i)):
                s = InputSlot(shape, index, self.device)
        else:
            s = InputSlot(shape, index, self.device)
        s.stream_i = stream_i
        ring.append(s)
        return s

    def _stage_ahead(self, nx: torch.Tensor, key, shape, current: InputSlot, ev_start,
                     main, ny: torch.Tensor | None = None, plan: bool = True) -> None:
        """Copy ids nx into a free slot and build its sparse plan there, on the slot's plan
        stream, concurrently with the step just enqueued (replayed from the slot's own
        plan graph once captured). plan=False: the copy only (plan_in_graph: the step
        before the batch's own builds its plan inside its graph)."""
        s = self._acquire_slot(shape, exclude=current, ahead=True)
        ps = self._stage_stream(s)
        ps.wait_event(ev_start)
        # torch.cuda.set_stream on the known streams instead of the torch.cuda.stream
        # context manager (~9 us per use: it looks the current stream up again)
        torch.cuda.set_stream(ps)
        try:
            # the ids and (ny) the labels in one launch where both are plain device copies
            yflat = ny.reshape(-1) if ny is not None else None
            if not hip_ops.batch_stage_copy(s.ids, nx, s.y if ny is not None else None, yflat):
                s.ids.copy_(nx, non_blocking=True)
                if ny is not None:
                    s.y.copy_(yflat, non_blocking=True)
            if nx.is_cuda:
                nx.record_stream(ps)
            s.y_key = None
            if ny is not None:  # the labels too: the step on this batch skips its copy
                if ny.is_cuda:
                    ny.record_stream(ps)
                s.y_key = self._xkey(ny)
            s.planned = plan
            if plan:
                self._plan_build_slot(s, ps)
            ev = self._slot_event(s)
            ev.record(ps)
        finally:
            torch.cuda.set_stream(main)
        s.ev = ev
        self._staged[key] = s

    def _stage_stream(self, s: InputSlot):
        """The plan stream of the next staged batch (slot s), in staging order. Every
        slot owns its buffers and plan scratch, so any plan stream may serve it; the slot's
        readers wait for its staging event, whichever stream recorded it."""
        s.stage_stream = self._slot_stream(self._stage_seq % max(1, self.n_plan_streams))
        self._stage_seq += 1
        return s.stage_stream

    def _slot_event(self, s: InputSlot):
        if s.done_ev is None:
            s.done_ev = torch.cuda.Event()
        return s.done_ev

    def _start_event(self):
        if self._ev_start is None:
            self._ev_start = torch.cuda.Event()
        return self._ev_start

    @staticmethod
    def _xkey(x):
        return (x.data_ptr(), tuple(x.shape), x.dtype, tuple(x.stride()), x.device)

    def _weights_version(self):
        mlp = self.model.mlp
        return (mlp[0].weight._version, mlp[3].weight._version)

    def _sync_weight_planes(self, force: bool = False) -> None:
        """Re-split the MLP weights' planes if the fp32 weights changed outside the trainer
        (load_state_dict, in-place ops on the Parameters: their version counters move).
        Writes through ``.data`` bypass the counters: call sync_weights() after those."""
        if self._wplanes is None:
            return
        ver = self._weights_version()
        if force or ver != self._wver:
            self._split_weights()
            self._wver = ver

    def sync_weights(self) -> None:
        """Tell the trainer the MLP weights were modified through ``.data``."""
        self._sync_weight_planes(force=True)

    def _after_step(self) -> None:
        """Host mirrors of what a step did on the device."""
        self.step_count += 1
        if self.deferred:
            self._dirty = True
        if self._pipe and self._bufs is not None and self._bufs.xps is not None:
            # this step's dW0 + MLP Adam are pending (they read its X planes)
            self._tail = (self._bufs, self._bufs.xp, self._bufs.xp_idx)

    def _pipe_state(self, slot: InputSlot):
        """(X plane buffer index of a step on `slot`, the pending tail or None). Each input
        slot writes X planes of its own, so in a slot ring the pending tail (the previous
        step, another slot) never holds the buffer the next gather writes: the steady state
        replays one graph per slot. A step on the slot of the pending tail (a repeated slot:
        no lookahead) writes the spare buffer (-1)."""
        if not self._pipe:
            return (0, None)
        idx, tail = slot.index, self._tail
        if tail is not None and tail[0].B == slot.shape[0] and tail[2] == idx:
            idx = -1
        return (idx, tail)

    def _xp_for(self, b: _Bufs, idx: int):
        """The bufset's X plane buffer number idx (allocated on first use, never inside a
        capture: the eager step that precedes each capture allocates it)."""
        xp = b.xps.get(idx)
        if xp is None:
            xp = b.xps[idx] = hip_ops.Planes(b.B, b.xp.cols, self.device, ones_col=True)
        return xp

    def _drain_tail(self) -> None:
        """Apply the pending weight-gradient tail now, on the current stream (eager)."""
        if self._tail is None:
            return
        tail, self._tail = self._tail, None
        with self._scratch.scope():
            self._tail_launch(tail)

    def _tail_launch(self, tail) -> None:
        """dW0 = dH1^T X (+ db0 from X's ones column) of the pending step and the Adam step of
        the MLP parameters with it, on the current stream. The step is the last completed one
        (the device counter step_done: read at run time, so a captured tail replays right)."""
        b, xp = tail[0], tail[1]
        gv = self.grad_views
        H1, W = b.h1.shape[1], b.dx.shape[1]
        self._gemm_planes(b.dh1p, xp, True, True, H1, W, b.B,
                          out=gv["mlp.0.weight"], last_col=gv["mlp.0.bias"])
        self._adam_dense(self.step_count, part="mlp", step_dev=self.step_done)

    def _graph_step(self, slot: InputSlot, mean_div: float, have: bool):
        if self.step_table.capacity < self.step_count + 2:
            self.step_table.ensure(max(self.step_count + 2, 2 * self.step_table.capacity))
        if self._graph_tab_version != self.step_table.version:
            torch.cuda.synchronize(self.device)  # none may still run when destroyed
            self._graphs.clear()  # they hold the old table's address
            self._graph_tab_version = self.step_table.version
        mlp = getattr(self.model, "mlp", None)
        drops = tuple(float(mlp[i].p) for i in (2, 5)) if mlp is not None else ()
        pipe = self._pipe_state(slot)
        nxt = self._next_plan
        key = (slot.shape, slot.index, mean_div, self.model.training, drops, have,
               pipe[0], None if pipe[1] is None else (pipe[1][0].B, pipe[1][2]),
               None if nxt is None else (nxt.shape, nxt.index))
        hit = self._graphs.get(key)
        if hit is None:
            # the real step (sizes every buffer), then the same launches captured
            loss = self._launch(slot.ids, slot.y, mean_div, have, plan=slot.plan, pipe=pipe)
            self._after_step()
            if len(self._graphs) < self.max_graphs:
                g = torch.cuda.CUDAGraph()
                with graph_capture(g, pool=live_pool(self), stream=self._capture_stream):
                    self._launch(slot.ids, slot.y, mean_div, have, plan=slot.plan, pipe=pipe)
                self._graphs[key] = (g, self._bufs)
                self.captures += 1
            return loss
        g, self._bufs = hit  # the buffer set the graph was captured with
        self._bufs.plan = slot.plan
        if self._bufs.xps is not None:  # the buffer the graph's gather writes
            self._bufs.xp = self._bufs.xps[pipe[0]]
            self._bufs.xp_idx = pipe[0]
        g.replay()
        self._after_step()
        return self._bufs.loss

    def _launch(self, x: torch.Tensor, y: torch.Tensor, mean_div: float,
                have_plan: bool = False, plan: hip_ops.SparsePlanBuffers | None = None,
                pipe=None) -> torch.Tensor:
        """Enqueue one step. Changes no host state: step-dependent values come from
        self.step_ctr (advanced on the device), so the launch sequence can be captured.
        plan: the batch's plan buffers (its input slot's; built here unless have_plan —
        built ahead on the plan stream by the previous steps' lookahead). pipe: the
        pipelined tail state (_pipe_state(slot), taken before the step; None: not
        pipelined — the replicated N > 1 path)."""
        B, F = x.shape
        rank, ws = world()
        b = self._buffers(B, F)
        b.plan = plan if plan is not None else b.plan_own
        piped = self._pipe and b.xps is not None and pipe is not None
        if piped:
            b.xp = self._xp_for(b, pipe[0])
            b.xp_idx = pipe[0]
        b.ev_tail = None
        y = y.reshape(-1)
        if y.dtype != torch.float32:
            y = y.float()
        y = y.contiguous()
        m = self.model
        E, bias = m.feature_embedding.weight.data, self.views.get("bias")
        w = m.linear.weight.data if self.kind != "IPNN" else None
        gv = self.grad_views
        step_hint = self.step_count + 1
        self._ev_wplanes = None
        ev_nplan = None  # FM plan_in_graph: the next batch's plan, joined before the tail
        if self._side is not None:
            # the sparse plan is only needed from the scatter on: build it on a side stream
            # while the catch-up (plan-free, from the ids) and the forward run here.
            # Capture order: in a HIP graph the first captured successor of a node continues
            # that node's hardware queue and the others start new queues; every fork / join
            # on the step's critical path costs ~5-12 us (rocprofv3 timelines) — so the
            # critical path is always enqueued before the branch that forks off it.
            main = hip_ops.current_stream()
            ev0 = torch.cuda.Event()
            ev0.record(main)  # x ready; previous step's plan users and Adam done
            ev_plan = torch.cuda.Event()

            def plan():
                if have_plan:
                    return  # built ahead: no fork
                self._side.wait_event(ev0)
                if not torch.cuda.is_current_stream_capturing():
                    x.record_stream(self._side)
                with torch.cuda.stream(self._side):
                    t_plan = self._mark("plan")
                    b.plan.build(x, self.V)
                    self._span("plan", t_plan)
                    ev_plan.record()

            if self.plan_first:
                plan()
            t = self._mark("catchup")
            if have_plan:
                # the plan built ahead lists the batch's unique rows: one launch over
                # them instead of the owner-marking pass + the id-driven catch-up
                hip_ops.adam_deferred_rows(E, self.m_E, self.v_E, w, self.m_w, self.v_w,
                                           self.last, b.plan, step_hint, self.step_table,
                                           self.betas, self.eps, self.weight_decay,
                                           step_dev=self.step_done)
            else:
                hip_ops.adam_deferred_catchup_ids(E, self.m_E, self.v_E, w, self.m_w,
                                                  self.v_w, self.last, x, self.rowmap,
                                                  self.step_done, self.step_table,
                                                  step_hint, self.betas, self.eps,
                                                  self.weight_decay)
            self._span("catchup", t)
            if piped and pipe[1] is not None:
                # the previous step's dW0 + MLP Adam beside this step's catch-up and gather
                # (one side list: the plan, when built in-step, follows it there)
                side = self._wgrad_stream
                side.wait_event(ev0)
                with torch.cuda.stream(side):
                    self._tail_launch(pipe[1])
                    b.ev_tail = torch.cuda.Event()
                    b.ev_tail.record()
            if not self.plan_first:
                plan()
            nxt = self._next_plan
            if nxt is not None and self.kind not in _MLP_KINDS:
                # FM (plan_in_graph): the next batch's plan on the side list, beside this
                # step's gather and scatter, joined before the step's tail: one graph launch
                # per step instead of a step graph and a plan graph
                self._side.wait_event(ev0)
                with torch.cuda.stream(self._side):
                    t_p = self._mark("plan")
                    nxt.plan.build(nxt.ids, self.V)
                    self._span("plan", t_p)
                    ev_nplan = torch.cuda.Event()
                    ev_nplan.record()
        else:
            t_plan = self._mark("plan")
            b.plan.build(x, self.V)  # rows of this batch (needed before the forward when deferred)
            self._span("plan", t_plan)
            if self.deferred:
                t = self._mark("catchup")
                hip_ops.adam_deferred_rows(E, self.m_E, self.v_E, w, self.m_w, self.v_w, self.last,
                                           b.plan, step_hint, self.step_table, self.betas,
                                           self.eps, self.weight_decay, step_dev=self.step_done)
                self._span("catchup", t)
        if self.kind == "FM":
            t = self._mark("gather")
            hip_ops.fm_forward(x, E, w, bias, want_sum=True, labels=y, mean_div=mean_div,
                               want_p=False, err_flag=self.err, out=b.fm)
            self._span("gather", t)
            gz = b.fm.gz
        else:
            gz = self._deepfm_forward_backward(x, y, b, E, w, bias, mean_div)
        # FM, one process: the bias gradient, the batch loss, the dense Adam and the step
        # counter in one launch at the end of the step (ctr_fm_step_tail)
        tail = self.kind == "FM" and ws == 1 and self._wplanes is None
        if self.kind == "FM" and not tail:  # MLP kinds: on the weight-gradient stream
            hip_ops.tensor_sum(gz, out=gv["bias"].view(1))
        if self._side is not None and not have_plan:
            hip_ops.current_stream().wait_event(ev_plan)  # the plan
        t = self._mark("scatter")
        sparse_rowmap = self.rowmap if (ws == 1 and not self.deferred) else None
        # one process, deferred Adam: the row sums are applied where they complete
        # (K >= 16: at C2 fused 48.5 vs separate 46.9 M ex/s, two alternating runs each, once
        # the host no longer paces the step; below 16 the separate apply pass is kept)
        fused = (ws == 1 and self.deferred and self._vec_ok and self.fuse_apply
                 and self.K >= self.fuse_apply_min_k)
        table = (E, self.m_E, self.v_E, w, self.m_w, self.v_w, self.last)
        apply_kw = dict(step_dev=self.step_cur, step_table=self.step_table, step=step_hint,
                        betas=self.betas, eps=self.eps, weight_decay=self.weight_decay)
        if self.kind == "IPNN":
            if fused:
                hip_ops.segment_sum_rows_adam(b.plan, b.dslot, None, table, **apply_kw,
                                              out=b.grad_rows, keep_sums=self.keep_grads)
            else:
                hip_ops.segment_sum_rows(b.plan, b.dslot, rowmap=sparse_rowmap, out=b.grad_rows)
        elif fused:
            hip_ops.fm_embedding_grad_adam(b.plan, F, gz, b.fm.sum_e, b.dx, table, **apply_kw,
                                           grad_rows=b.grad_rows, grad_lin=b.grad_lin,
                                           keep_sums=self.keep_grads)
        else:
            hip_ops.fm_embedding_grad(b.plan, F, E, gz, b.fm.sum_e, b.dx, sparse_rowmap,
                                      grad_rows=b.grad_rows, grad_lin=b.grad_lin)
        self._span("scatter", t)
        if self.kind in _MLP_KINDS:  # captured after the scatter: see the capture-order note
            self._weight_grads(b, gz)
        if self.kind == "FM" and not tail:  # MLP kinds: on the weight-gradient stream
            hip_ops.tensor_sum(b.fm.loss_elem, scale=1.0 / B, out=b.loss)
        grad_rows, grad_lin, plan = b.grad_rows, (b.grad_lin if w is not None else None), b.plan
        if ws > 1:
            self._join_wgrad()  # the exchange all-reduces the dense gradient
            grad_rows, grad_lin = self._exchange(b)
            plan = b.gplan
        t = self._mark("adam")
        if fused:
            pass  # applied inside the segmented sums above
        elif self.deferred:
            hip_ops.adam_deferred_rows(E, self.m_E, self.v_E, w, self.m_w, self.v_w, self.last,
                                       plan, step_hint, self.step_table, self.betas,
                                       self.eps, self.weight_decay, grad_rows=grad_rows,
                                       grad_lin=grad_lin, step_dev=self.step_cur)
        else:
            hip_ops.adam_embedding(E, self.m_E, self.v_E, w, self.m_w, self.v_w, self.rowmap,
                                   grad_rows, grad_lin, step_hint, self.lr, self.betas,
                                   self.eps, self.weight_decay, step_dev=self.step_cur,
                                   table=self.step_table)
        self._span("adam", t)
        if ev_nplan is not None:
            hip_ops.current_stream().wait_event(ev_nplan)
        # the dense Adam where the dense gradient completes: on the weight-gradient stream
        # at one process (beside the embedding apply), after the exchange otherwise
        if tail:
            t = self._mark("adam")
            hip_ops.fm_step_tail(b.fm.loss_elem, gz, 1.0 / B, b.loss, gv["bias"].view(1),
                                 self.flat, self.flat_grad, self.m_flat, self.v_flat,
                                 self.step_table, step_hint, self.step_ctr, self.betas,
                                 self.eps, self.weight_decay, loss_sum=self.loss_sum)
            self._span("adam", t)
            return b.loss
        wg = self._wgrad_stream if ws == 1 else None
        if wg is None:
            self._join_wgrad()
        with torch.cuda.stream(wg) if wg is not None else _nullctx():
            # pipelined: the FM bias now (the next step's gather reads it), the MLP at the
            # start of the next step (_tail_launch)
            self._adam_dense(step_hint, part="bias" if piped else "all")
        self._join_wgrad()
        hip_ops.step_end(self.step_ctr, b.loss, self.loss_sum)
        return b.loss

    def _adam_dense(self, step_hint: int, part: str = "all", step_dev=None) -> None:
        """The flat dense parameters' Adam step; the MLP weights' planes are rewritten with
        the updated values (the next step's GEMM operands) — by the Adam kernel itself when
        a weight's row length is a multiple of 4, by a split pass after it otherwise.
        part: "all", "bias" (the FM bias alone: the flat buffer ahead of mlp.0.weight) or
        "mlp" (from mlp.0.weight on) — elementwise, so the two parts are bitwise the one
        launch. step_dev: the device step counter to read (default: the step in flight)."""
        lo = 0
        hi = self.flat.numel()
        if part != "all" and "mlp.0.weight" in self.offsets:
            cut = self.offsets["mlp.0.weight"]
            lo, hi = (0, cut) if part == "bias" else (cut, hi)
        if lo == hi:
            return
        planes, resplit = [], []
        if self._wplanes is not None and part != "bias":
            for name, pl in zip(("mlp.0.weight", "mlp.3.weight"), self._wplanes):
                if pl.cols % 4 == 0 and (self.offsets[name] - lo) % 4 == 0:
                    planes.append((self.offsets[name] - lo, pl))
                else:
                    resplit.append((name, pl))
        hip_ops.adam_dense(self.flat[lo:hi], self.flat_grad[lo:hi], self.m_flat[lo:hi],
                           self.v_flat[lo:hi], step_hint, self.lr, self.betas, self.eps,
                           self.weight_decay,
                           step_dev=self.step_cur if step_dev is None else step_dev,
                           table=self.step_table, planes=planes or None)
        for name, pl in resplit:
            hip_ops.split_planes(self.views[name], out=pl)

    def _deepfm_forward_backward(self, x, y, b: _Bufs, E, w, bias, mean_div):
        """The MLP part of DeepFM / InnerPNN (p_model.py:276-293,322 and 185-200) on
        pre-split planes: 6 GEMMs per step, every operand read in the orientation its
        producer wrote it (the transposed products of the backward by the GEMM's transpose
        read), no transposed copy anywhere."""
        mlp, gv, vw = self.model.mlp, self.grad_views, self.views
        training = self.model.training
        p0 = float(mlp[2].p) if training else 0.0
        p1 = float(mlp[5].p) if training else 0.0
        B = x.shape[0]
        H1, H2 = b.h1.shape[1], b.h2.shape[1]
        W = b.xp.cols
        w0p, w1p = self._wplanes
        # dropout stream of this step: (completed steps) << 32 is added on the device.
        # The counter is the GLOBAL-batch element index (rank r's local row m is global row
        # r*B + m), so N ranks draw exactly the masks one process draws on the global batch
        # (independent masks per rank; tests/test_gpu_sharded.py checks the equality)
        rank, ws = world()
        off1 = rank * B * H1
        off2 = ws * B * H1 + rank * B * H2
        t = self._mark("gather")
        if self.kind == "IPNN":  # cat = flat(E[x]) ++ pairwise inner products, as planes
            X = hip_ops.ipnn_forward(x, E, out=None, err_flag=self.err, planes=b.xp)
            z_fm = b.zero
        elif b.fm.emb_out is None:  # gather + FM, the MLP input written as its planes
            hip_ops.fm_forward_planes(x, E, w, bias, b.xp, b.fm.z, b.fm.sum_e, err_flag=self.err)
            X, z_fm = None, b.fm.z
        else:
            fm = hip_ops.fm_forward(x, E, w, bias, want_sum=True, want_emb=True, want_p=False,
                                    err_flag=self.err, out=b.fm)
            X, z_fm = fm.emb_out, fm.z
        if X is not None:
            hip_ops.split_planes(X, out=b.xp)
        self._span("gather", t)
        if getattr(b, "ev_tail", None) is not None:  # the previous step's MLP Adam
            hip_ops.current_stream().wait_event(b.ev_tail)
        # Linear(F*K,300)+ReLU+Dropout: H1 (fp32 for the mask, planes for the next GEMMs)
        self._gemm_planes(b.xp, w0p, False, False, B, H1, W, out=b.h1, out_planes=b.h1p,
                          epi=hip_ops.EPI_BIAS_RELU_DROP if p0 > 0 else hip_ops.EPI_BIAS_RELU,
                          bias=vw["mlp.0.bias"], drop_p=p0, seed=self.seed, offset=off1,
                          step_dev=self.step_done)
        self._gemm_planes(b.h1p, w1p, False, False, B, H2, H1, out=b.h2,
                          epi=hip_ops.EPI_BIAS_RELU_DROP if p1 > 0 else hip_ops.EPI_BIAS_RELU,
                          bias=vw["mlp.3.bias"], drop_p=p1, seed=self.seed, offset=off2,
                          step_dev=self.step_done)
        head = hip_ops.deepfm_head(b.h2, vw["mlp.6.weight"], vw["mlp.6.bias"], z_fm, y,
                                   mean_div=mean_div, drop_scale=1.0 / (1.0 - p1), out=b.head,
                                   dh_planes=b.dh2p)
        gz = head["gz"]
        b.ev_head = torch.cuda.Event()
        b.ev_head.record()
        # Linear(300,200): dH1 = (dH2 @ W1) masked by Dropout+ReLU of layer 1
        # (planes only: dX and dW0 read dH1 as planes, nothing reads an fp32 copy)
        self._gemm_planes(b.dh2p, w1p, False, True, B, H1, H2, out=None, out_planes=b.dh1p,
                          epi=hip_ops.EPI_GRAD_MASK, aux=b.h1, scale=1.0 / (1.0 - p0))
        # Linear(F*K,300): dX = dH1 @ W0, the MLP-input gradient the scatter needs
        self._gemm_planes(b.dh1p, w0p, False, True, B, W, H1, out=b.dx)
        if self.kind == "IPNN":  # per-slot embedding gradients through the pair products
            hip_ops.ipnn_backward(x, E, b.dx, out=b.dslot)
        b.ev_dx = torch.cuda.Event()
        b.ev_dx.record()
        return gz

    def _split_weights(self) -> None:
        """The MLP weights' bf16 planes, re-split from the fp32 parameters every step."""
        w0p, w1p = self._wplanes
        hip_ops.split_planes(self.views["mlp.0.weight"], out=w0p)
        hip_ops.split_planes(self.views["mlp.3.weight"], out=w1p)

    def _weight_grads(self, b: _Bufs, gz) -> None:
        """The dense-parameter gradients, needed only by the dense Adam at the end of the
        step, on the side stream: from the head on (under dH1 / dX) one launch pair of
        column sums (batch loss, FM bias, mlp.6) and dW1 with db1 (ones-column GEMM), from
        dX on (under the scatter and the embedding Adam) db0 and dW0. Enqueued after the
        scatter so that, in the captured graph, the dH1 -> dX -> scatter chain keeps one
        queue. Measured alternatives (rocprofv3 timelines, C3): forking everything from dH1
        (side kernels dispatched after dX has filled the CUs: +40 us), dW0 from dH1 (it then
        takes the CUs ahead of the scatter chain: +25 us)."""
        gv, B = self.grad_views, b.B
        side = self._wgrad_stream
        H1, H2, W = b.h1.shape[1], b.h2.shape[1], b.dx.shape[1]
        if side is not None:
            side.wait_event(b.ev_head)
        with torch.cuda.stream(side) if side is not None else _nullctx():
            jobs = [(b.fm.loss_elem.view(B, 1), None, b.loss, 1.0 / B)]  # batch mean BCE
            if "bias" in gv:  # DeepFM's FM bias: sum gz
                jobs.append((gz.view(B, 1), None, gv["bias"].view(1)))
            # Linear(200,1): dW = gz^T H2, db = sum gz
            jobs += [(b.h2, gz, gv["mlp.6.weight"].view(-1)),
                     (gz.view(B, 1), None, gv["mlp.6.bias"].view(1))]
            # Linear(300,200): dW1 = dH2^T H1, db1 = colsum dH2 (H1's ones column)
            self._gemm_planes(b.dh2p, b.h1p, True, True, H2, H1, B,
                              out=gv["mlp.3.weight"], last_col=gv["mlp.3.bias"])
            nxt = self._next_plan
            if nxt is not None:  # the next batch's plan, beside dX (plan_in_graph)
                t = self._mark("plan")
                nxt.plan.build(nxt.ids, self.V)
                self._span("plan", t)
            if side is not None:  # from dX on
                side.wait_event(b.ev_dx)
            # the column-sum pair here, ahead of dW0: seg_chunk takes the CUs before dW0
            # does (measured at C3: db0's column sum moved before the dX fork let dW0 and
            # seg_chunk start together, seg_chunk 38 -> 106 us, the step +20 us); and
            # Linear(F*K,300)'s db0 = colsum dH1 comes out of dW0 = dH1^T X as the ones
            # column of X
            hip_ops.colsum_multi(jobs)
            if not (self._pipe and b.xps is not None):  # pipelined: at the next step's start
                self._gemm_planes(b.dh1p, b.xp, True, True, H1, W, B,
                                  out=gv["mlp.0.weight"], last_col=gv["mlp.0.bias"])

    def _join_wgrad(self) -> None:
        """The dense-parameter gradients are complete on the current stream after this."""
        if self._wgrad_stream is not None:
            hip_ops.current_stream().wait_stream(self._wgrad_stream)

    def _exchange(self, b: _Bufs):
        """Sum embedding-row gradients over ranks (deterministic, identical everywhere)."""
        allreduce_sum_(self.flat_grad, self.group)
        allreduce_sum_(b.loss, self.group)
        b.loss.div_(world()[1])
        U = b.plan.num_unique_host()
        rows_all, vals_all, lin_all = allgather_sparse_rows(b.plan.unique_rows, b.grad_rows,
                                                            b.grad_lin, U, self.group)
        b.gplan.build(rows_all, self.V)
        hip_ops.segment_sum_rows(b.gplan, vals_all, lin_all,
                                 rowmap=None if self.deferred else self.rowmap, out=b.g_rows,
                                 out_lin=b.g_lin)
        return b.g_rows, b.g_lin

    def check_errors(self) -> None:
        """Raise IndexError if any kernel saw a feature id outside [0, V). Syncs."""
        hip_ops.check_index_error(self.err)
