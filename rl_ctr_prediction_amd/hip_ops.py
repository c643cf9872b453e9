"""Tensor-level wrappers over the libctr_hip.so C ABI.

PyTorch only provides device memory and the current HIP stream here; every computation
is a kernel of libctr_hip.so. Inputs must already be on a ROCm device: a CPU tensor is
an error, never a silent fallback.
"""
from __future__ import annotations

import contextlib
import os
import ctypes
import threading
from dataclasses import dataclass

import torch

from ._lib import (CTR_EFLAG_CAPACITY, CTR_EFLAG_INDEX, CTR_IDX_I32, CTR_IDX_I64, EPI_BIAS, EPI_BIAS_RELU,
                   EPI_BIAS_RELU_DROP, EPI_GRAD_MASK, EPI_NONE, PlanesDesc, PlaneViewDesc, SparsePlan,
                   lib)

__all__ = [
    "embedding_gather", "fm_forward", "fm_forward_planes", "bce_sigmoid", "deepfm_head", "gemm", "linear",
    "tensor_sum", "colsum", "transpose", "Planes", "split_planes", "gemm_planes", "SparsePlanBuffers", "fm_embedding_grad", "segment_sum_rows",
    "fm_embedding_grad_adam", "segment_sum_rows_adam",
    "rows_to_dense", "adam_dense", "fm_step_tail", "adam_embedding", "adam_scalars", "feature_embedding",
    "AdamStepTable", "adam_deferred_rows", "adam_deferred_flush", "adam_deferred_catchup_ids",
    "step_begin", "step_end", "ids_add_", "shard_pack_ids", "shard_runs_copy",
    "softmax_rows", "pg_discount_norm", "pg_loss_grad", "pg_vt_mean", "pg_loss_grad_global", "check_index_error", "Workspace",
    "EPI_NONE", "EPI_BIAS", "EPI_BIAS_RELU", "EPI_BIAS_RELU_DROP", "EPI_GRAD_MASK",
]


# ----------------------------------------------------------------------- plumbing ----
def _dev(t: torch.Tensor, name: str = "tensor") -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} is on {t.device}: the HIP hot path needs ROCm device "
                           "tensors (there is no CPU fallback)")
    return t


def _f32(t: torch.Tensor, name: str) -> torch.Tensor:
    _dev(t, name)
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    return t


def _p(t):
    return None if t is None else t.data_ptr()


_cuda_device = torch._C._cuda_getDevice
_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_stream = torch._C._cuda_getCurrentStream


def _stream() -> int:
    """The current stream's HIP handle, without torch.cuda.current_stream()'s Python-level
    device lookup (~4 us a call: the host paces C2's steps)."""
    return _raw_stream(_cuda_device())


def current_stream() -> torch.cuda.Stream:
    """torch.cuda.current_stream() for the current device, minus its device-index lookup."""
    d = _cur_stream(_cuda_device())
    return torch.cuda.Stream(stream_id=d[0], device_index=d[1], device_type=d[2])


def _idx(t: torch.Tensor, name: str = "idx") -> tuple[torch.Tensor, int]:
    _dev(t, name)
    if t.dtype == torch.int64:
        it = CTR_IDX_I64
    elif t.dtype == torch.int32:
        it = CTR_IDX_I32
    else:
        raise TypeError(f"{name}: feature ids must be int64 or int32, got {t.dtype}")
    return t.contiguous(), it


class Workspace:
    """Grow-only scratch buffers of ONE owner, one per (device, stream) inside it: kernels
    on one stream are ordered, so consecutive ops of the owner can share a buffer. A buffer
    outgrown is retired, never freed: HIP graphs captured earlier still hold its address.

    Every trainer (and PolicyGradient) owns a Workspace and enters it (``with ws.scope():``)
    around the launches it enqueues or captures, so no captured graph references scratch
    that another object's launches also use — two objects' streams may share a HIP handle
    (torch hands streams out of a small pool round-robin) without sharing scratch. Calls
    made outside any scope (one-off op calls, tests) use the process-wide default owner."""

    _default: "Workspace | None" = None
    _tls = threading.local()

    def __init__(self):
        self._pool: dict = {}
        self._retired: list = []

    @contextlib.contextmanager
    def scope(self):
        stack = getattr(Workspace._tls, "stack", None)
        if stack is None:
            stack = Workspace._tls.stack = []
        stack.append(self)
        try:
            yield self
        finally:
            stack.pop()

    @classmethod
    def current(cls) -> "Workspace":
        stack = getattr(cls._tls, "stack", None)
        if stack:
            return stack[-1]
        if cls._default is None:
            cls._default = Workspace()
        return cls._default

    def buffer(self, nbytes: int, device: torch.device) -> torch.Tensor | None:
        if nbytes <= 0:
            return None
        key = (device.index, _stream())
        buf = self._pool.get(key)
        if buf is None or buf.numel() < nbytes:
            if buf is not None:
                self._retired.append(buf)
            buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            self._pool[key] = buf
        return buf

    def buffers(self) -> list:
        """Every buffer this owner holds (tests: owners never share one)."""
        return list(self._pool.values()) + list(self._retired)

    @classmethod
    def get(cls, nbytes: int, device: torch.device) -> torch.Tensor | None:
        """Scratch of nbytes on the current stream, from the current owner."""
        return cls.current().buffer(nbytes, device)


def check_index_error(err_flag: torch.Tensor) -> None:
    """Raise like nn.Embedding does when a kernel saw an id outside [0, V). Syncs."""
    v = int(err_flag.item())
    if v & CTR_EFLAG_CAPACITY:  # a library invariant broke (the host sizes the capacity)
        err_flag.zero_()
        raise RuntimeError("row-sharded exchange: a run exceeded its capacity")
    if v & CTR_EFLAG_INDEX:
        err_flag.zero_()
        raise IndexError("index out of range in self")


# ------------------------------------------------------------------------ forward ----
def embedding_gather(table: torch.Tensor, idx: torch.Tensor, err_flag=None,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    _f32(table, "table")
    idx, it = _idx(idx)
    V, K = table.shape
    if out is None:
        out = torch.empty(*idx.shape, K, dtype=torch.float32, device=table.device)
    elif out.numel() < idx.numel() * K or not out.is_contiguous():
        raise ValueError("embedding_gather: out must be contiguous with idx.numel() * K floats")
    lib.ctr_embedding_gather(_p(table), V, K, _p(idx), it, idx.numel(), _p(out), _p(err_flag),
                             _stream())
    return out


@dataclass
class FMForward:
    z: torch.Tensor
    sum_e: torch.Tensor | None
    emb_out: torch.Tensor | None
    p: torch.Tensor | None
    loss_elem: torch.Tensor | None
    gz: torch.Tensor | None


def fm_forward(idx: torch.Tensor, emb: torch.Tensor, lin: torch.Tensor, bias: torch.Tensor, *,
               want_sum: bool = True, want_emb: bool = False, labels: torch.Tensor | None = None,
               mean_div: float | None = None, want_p: bool = True, err_flag=None,
               out: FMForward | None = None) -> FMForward:
    """Fused gather + FM second order + linear term (+ BCE head when labels are given)."""
    idx, it = _idx(idx)
    B, F = idx.shape
    _f32(emb, "feature_embedding.weight")
    _f32(lin, "linear.weight")
    _f32(bias, "bias")
    V, K = emb.shape
    dev = emb.device
    if out is None:
        e = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        out = FMForward(z=e(B), sum_e=e(B, K) if want_sum else None,
                        emb_out=e(B, F * K) if want_emb else None,
                        p=e(B) if want_p else None,
                        loss_elem=e(B) if labels is not None else None,
                        gz=e(B) if labels is not None else None)
    if labels is not None:
        _f32(labels, "labels")
        mean_div = float(B if mean_div is None else mean_div)
    lib.ctr_fm_forward(_p(idx), it, B, F, K, V, _p(emb), _p(lin), _p(bias), _p(out.z),
                       _p(out.sum_e), _p(out.emb_out), _p(labels), float(mean_div or 1.0),
                       _p(out.p), _p(out.loss_elem), _p(out.gz), _p(err_flag), _stream())
    return out


def fm_forward_planes(idx: torch.Tensor, emb: torch.Tensor, lin: torch.Tensor,
                      bias: torch.Tensor, x_planes: "Planes", z: torch.Tensor,
                      sum_e: torch.Tensor, err_flag=None) -> None:
    """DeepFM's FM part (z, sum_e) with the flattened embeddings written as the MLP input's
    three bf16 planes (no fp32 copy): ctr_fm_forward_planes."""
    idx, it = _idx(idx)
    B, F = idx.shape
    _f32(emb, "feature_embedding.weight")
    _f32(lin, "linear.weight")
    V, K = emb.shape
    if (x_planes.rows, x_planes.cols) != (B, F * K):
        raise ValueError(f"fm_forward_planes: planes must be [{B}, {F * K}]")
    lib.ctr_fm_forward_planes(_p(idx), it, B, F, K, V, _p(emb), _p(lin), _p(bias), _p(z),
                              _p(sum_e), x_planes.desc, _p(err_flag), _stream())


def fm_forward_planes_ok(K: int, F: int) -> bool:
    return K % 4 == 0 and 64 % (K // 4 or 1) == 0 and K <= 256 and F <= 64


def bce_sigmoid(z: torch.Tensor, labels: torch.Tensor, mean_div: float | None = None):
    _f32(z, "z")
    _f32(labels, "labels")
    B = z.numel()
    p, loss, gz = (torch.empty_like(z) for _ in range(3))
    lib.ctr_bce_sigmoid(_p(z), _p(labels), B, float(B if mean_div is None else mean_div), _p(p),
                        _p(loss), _p(gz), _stream())
    return p, loss, gz


def deepfm_head(h, w_out, b_out, z_fm, labels=None, mean_div=None, drop_scale=1.0, out=None,
                dh_planes: "Planes | None" = None):
    """dh_planes: also write dh_pre as its three bf16 planes (ctr_deepfm_head_planes)."""
    _f32(h, "h")
    B, H = h.shape
    dev = h.device
    if out is None:
        e = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        out = dict(z=e(B), p=e(B), loss_elem=e(B) if labels is not None else None,
                   gz=e(B) if labels is not None else None,
                   dh_pre=e(B, H) if labels is not None else None)
    if dh_planes is not None:
        if labels is None or (dh_planes.rows, dh_planes.cols) != (B, H):
            raise ValueError(f"deepfm_head: dh_planes needs labels and [{B}, {H}] planes")
        lib.ctr_deepfm_head_planes(_p(h), B, H, _p(w_out), _p(b_out), _p(z_fm), _p(labels),
                                   float(B if mean_div is None else mean_div), float(drop_scale),
                                   _p(out["z"]), _p(out["p"]), _p(out["loss_elem"]),
                                   _p(out["gz"]), _p(out["dh_pre"]), dh_planes.desc, _stream())
        return out
    lib.ctr_deepfm_head(_p(h), B, H, _p(w_out), _p(b_out), _p(z_fm), _p(labels),
                        float(B if mean_div is None else mean_div), float(drop_scale),
                        _p(out["z"]), _p(out["p"]), _p(out["loss_elem"]), _p(out["gz"]),
                        _p(out["dh_pre"]), _stream())
    return out


# --------------------------------------------------------------------------- GEMM ----
GEMM_AUTO, GEMM_EXACT_F32, GEMM_SPLIT_BF16 = 0, 1, 2  # enum ctr_gemm_algo


def gemm(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False, trans_b: bool = False, *,
         epi: int = EPI_NONE, bias=None, aux=None, scale: float = 1.0, drop_p: float = 0.0,
         seed: int = 0, offset: int = 0, step_dev: torch.Tensor | None = None,
         out: torch.Tensor | None = None, algo: int = GEMM_AUTO) -> torch.Tensor:
    """C = op(a) @ op(b) on the MFMA units with a fused epilogue (see include/ctr_hip.h):
    algo GEMM_EXACT_F32 (fp32 MFMA) or GEMM_SPLIT_BF16 (three-plane bf16 split, fp32
    accurate); GEMM_AUTO = the library default. step_dev (device int32): the dropout stream
    of that step (offset += step << 32)."""
    _f32(a, "A")
    _f32(b, "B")
    M, K = (a.shape[1], a.shape[0]) if trans_a else a.shape
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else b.shape
    if K != Kb:
        raise ValueError(f"gemm: inner dims differ ({K} vs {Kb})")
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=a.device)
    else:
        _f32(out, "out")
        if tuple(out.shape) != (M, N):
            raise ValueError("gemm: bad out shape")
    if aux is not None:
        _f32(aux, "aux")
    nbytes = lib.ctr_gemm_f32_ex_workspace_bytes(int(algo), int(trans_a), int(trans_b), M, N, K)
    ws = Workspace.get(nbytes, a.device)
    lib.ctr_gemm_f32_ex(int(algo), int(trans_a), int(trans_b), M, N, K, _p(a), a.stride(0), _p(b),
                        b.stride(0), _p(out), out.stride(0), int(epi), _p(bias), _p(aux),
                        aux.stride(0) if aux is not None else 0, float(scale), float(drop_p),
                        int(seed) & (2**64 - 1), int(offset) & (2**64 - 1), _p(step_dev), _p(ws),
                        0 if ws is None else ws.numel(), _stream())
    return out


class Planes:
    """An fp32 matrix [rows, cols] held as its exact three-plane bf16 split (ctr_planes):
    one bf16 tensor [3, rows_pad, cols_pad], both extents padded to multiples of 32 with
    zeros (allocated zeroed; producers write only the valid region, so the pad stays zero).
    x = x0 + (x1 + x2) recovers every fp32 element exactly (to_float)."""

    def __init__(self, rows: int, cols: int, device, pad: int = 32, ones_col: bool = False):
        self.rows, self.cols = int(rows), int(cols)
        self.rows_pad = -(-max(self.rows, 1) // pad) * pad
        self.cols_pad = -(-max(self.cols + int(ones_col), 1) // pad) * pad
        self.t = torch.zeros(3, self.rows_pad, self.cols_pad, dtype=torch.bfloat16, device=device)
        # ones_col: column `cols` (in the padding) holds 1.0 — exact in plane 0, zero in the
        # others — so a GEMM reading this matrix as B with N = cols + 1 also returns the
        # column sums of A (gemm_planes(last_col=...)); GEMMs with K = cols never read it.
        self.ones_col = bool(ones_col)
        if ones_col:
            self.t[0, :self.rows, self.cols] = 1.0
        self.desc = PlanesDesc(self.t.data_ptr(), self.cols_pad, self.rows_pad * self.cols_pad,
                               self.rows_pad, self.cols_pad)

    @property
    def device(self):
        return self.t.device

    def to_float(self) -> torch.Tensor:
        """The fp32 matrix (x0 + (x1 + x2), exact)."""
        p = self.t[:, :self.rows, :self.cols].float()
        return p[0] + (p[1] + p[2])


def split_planes(src: torch.Tensor, out: Planes | None = None) -> Planes:
    """The exact three-plane bf16 split of an fp32 [rows, cols] matrix (row-contiguous)."""
    _dev(src, "src")
    if src.dtype != torch.float32 or src.dim() != 2 or (src.numel() and src.stride(1) != 1):
        raise ValueError("split_planes: src must be a float32 [rows, cols] row-contiguous matrix")
    R, Cn = src.shape
    if out is None:
        out = Planes(R, Cn, src.device)
    elif out.rows != R or out.cols != Cn:
        raise ValueError(f"split_planes: out planes are [{out.rows}, {out.cols}], src [{R}, {Cn}]")
    lib.ctr_split_planes(_p(src), R, Cn, src.stride(0) if R > 1 else Cn, out.desc, _stream())
    return out


def gemm_planes(a: Planes, b: Planes, a_rc: bool, b_rc: bool, *, out: torch.Tensor | None = None,
                out_planes: Planes | None = None, epi: int = EPI_NONE, bias=None, aux=None,
                scale: float = 1.0, drop_p: float = 0.0, seed: int = 0, offset: int = 0,
                step_dev: torch.Tensor | None = None,
                last_col: torch.Tensor | None = None) -> torch.Tensor | None:
    """C = A.B on pre-split planes (ctr_gemm_planes). a_rc: A holds A^T ([K, M]); b_rc: B holds
    B itself ([K, N]) rather than the nn.Linear form [N, K]. Writes `out` (fp32 [M, N]) and/or
    `out_planes` (the planes of the epilogue's result).
    last_col ([M]): B (b_rc, built with ones_col) gets its ones column appended, and the
    extra result column — the row sums of A^T's rows, i.e. colsum of the stored A — lands
    here (ctr_gemm_planes_lastcol)."""
    M, K = (a.cols, a.rows) if a_rc else (a.rows, a.cols)
    N, Kb = (b.cols, b.rows) if b_rc else (b.rows, b.cols)
    if K != Kb:
        raise ValueError(f"gemm_planes: inner dims differ ({K} vs {Kb})")
    if last_col is not None:
        _f32(last_col, "last_col")
        if not (b_rc and b.ones_col) or out is None or out_planes is not None:
            raise ValueError("gemm_planes: last_col needs b_rc planes with ones_col and an fp32 out")
        if last_col.numel() != M or not last_col.is_contiguous():
            raise ValueError(f"gemm_planes: last_col must be {M} contiguous floats")
        if tuple(out.shape) != (M, N) or (out.numel() and out.stride(1) != 1):
            raise ValueError(f"gemm_planes: out must be [{M}, {N}]")
        nbytes = lib.ctr_gemm_planes_workspace_bytes(int(a_rc), 1, M, N + 1, K)
        ws = Workspace.get(nbytes, a.device)
        lib.ctr_gemm_planes_lastcol(int(a_rc), 1, M, N + 1, K, a.desc, b.desc, _p(out),
                                    out.stride(0), None, int(epi), _p(bias), None, 0,
                                    float(scale), 0.0, 0, 0, None, _p(last_col), _p(ws),
                                    0 if ws is None else ws.numel(), _stream())
        return out
    if out is None and out_planes is None:
        out = torch.empty(M, N, dtype=torch.float32, device=a.device)
    if out is not None:
        _f32(out, "out")
        if tuple(out.shape) != (M, N):
            raise ValueError(f"gemm_planes: out must be [{M}, {N}]")
    if out_planes is not None and (out_planes.rows, out_planes.cols) != (M, N):
        raise ValueError(f"gemm_planes: out_planes must be [{M}, {N}]")
    if aux is not None:
        _f32(aux, "aux")
    nbytes = lib.ctr_gemm_planes_workspace_bytes(int(a_rc), int(b_rc), M, N, K)
    ws = Workspace.get(nbytes, a.device)
    lib.ctr_gemm_planes(int(a_rc), int(b_rc), M, N, K, a.desc, b.desc, _p(out),
                        out.stride(0) if out is not None else 0,
                        out_planes.desc if out_planes is not None else None, int(epi), _p(bias),
                        _p(aux), aux.stride(0) if aux is not None else 0, float(scale),
                        float(drop_p), int(seed) & (2**64 - 1), int(offset) & (2**64 - 1),
                        _p(step_dev), _p(ws), 0 if ws is None else ws.numel(), _stream())
    return out


def gemm_planes_config(a_rc: bool, b_rc: bool, M: int, N: int, K: int) -> dict:
    """The tiling ctr_gemm_planes picks for a shape (tuning / tests)."""
    import ctypes
    v = [ctypes.c_int(0) for _ in range(4)]
    lib.ctr_gemm_planes_config(int(a_rc), int(b_rc), M, N, K, *(ctypes.byref(x) for x in v))
    return dict(tile=v[0].value, splits=v[1].value, bm=v[2].value, bn=v[3].value)


def linear(x, weight, bias, *, relu=False, drop_p=0.0, seed=0, offset=0, step_dev=None, out=None):
    """nn.Linear (+ReLU +Dropout) forward: x @ weight.T + bias, fused epilogue."""
    if relu:
        epi = EPI_BIAS_RELU_DROP if drop_p > 0 else EPI_BIAS_RELU
    else:
        epi = EPI_BIAS
    return gemm(x, weight, False, True, epi=epi, bias=bias, drop_p=drop_p, seed=seed,
                offset=offset, step_dev=step_dev, out=out)


def tensor_sum(x: torch.Tensor, scale: float = 1.0, out=None) -> torch.Tensor:
    _f32(x, "x")
    if out is None:
        out = torch.empty(1, dtype=torch.float32, device=x.device)
    ws = Workspace.get(lib.ctr_reduce_workspace_bytes(x.numel(), 1), x.device)
    lib.ctr_sum_f32(_p(x), x.numel(), float(scale), _p(out), _p(ws), ws.numel(), _stream())
    return out


def colsum_multi(jobs) -> None:
    """Several colsum() calls in one launch pair: jobs = [(X [M,N], row_w or None, out [N]
    [, scale])]; each out is bitwise what colsum(X, row_w, scale, out=out) writes."""
    from ._lib import ColsumJob
    arr = (ColsumJob * len(jobs))()
    for i, job in enumerate(jobs):
        X, row_w, out = job[:3]
        scale = float(job[3]) if len(job) > 3 else 1.0
        _f32(X, "X")
        if X.dim() != 2 or out.numel() != X.shape[1]:
            raise ValueError("colsum_multi: X must be [M, N] and out N elements")
        arr[i] = ColsumJob(_p(X), X.shape[0], X.shape[1], X.stride(0), _p(row_w), scale, _p(out))
    nbytes = lib.ctr_colsum_multi_workspace_bytes(len(jobs), arr)
    ws = Workspace.get(nbytes, jobs[0][0].device)
    lib.ctr_colsum_multi_f32(len(jobs), arr, _p(ws), ws.numel(), _stream())


def colsum(X: torch.Tensor, row_w: torch.Tensor | None = None, scale: float = 1.0,
           out=None) -> torch.Tensor:
    _f32(X, "X")
    M, N = X.shape
    if out is None:
        out = torch.empty(N, dtype=torch.float32, device=X.device)
    ws = Workspace.get(lib.ctr_reduce_workspace_bytes(M, N), X.device)
    lib.ctr_colsum_f32(_p(X), M, N, X.stride(0), _p(row_w), float(scale), _p(out), _p(ws),
                       ws.numel(), _stream())
    return out


def transpose(src: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """out[c, r] = src[r, c] (bit-exact; src rows may be strided, out contiguous)."""
    _dev(src, "src")
    if src.dtype != torch.float32:
        raise TypeError(f"src: expected float32, got {src.dtype}")
    R, Cn = src.shape
    if src.numel() and src.stride(1) != 1:
        raise ValueError("transpose: src rows must be contiguous")
    if R > 1 and src.stride(0) < Cn:  # a stride-0 / overlapping row view (x.expand(R, C))
        raise ValueError("transpose: src rows must not overlap (stride(0) >= columns)")
    if out is None:
        out = torch.empty(Cn, R, dtype=torch.float32, device=src.device)
    if tuple(out.shape) != (Cn, R) or (out.numel() and out.stride(1) != 1):
        raise ValueError(f"transpose: out must be a row-contiguous [{Cn}, {R}] tensor")
    lib.ctr_transpose_f32(_p(src), R, Cn, src.stride(0) if R > 1 else Cn, _p(out), max(out.stride(0), R),
                          _stream())
    return out


# ---------------------------------------------------------------- scatter-add -------
# CTR_PLAN_COLS=0: the LSD plan for [B, F] ids too (A/B)
_PLAN_COLS = os.environ.get("CTR_PLAN_COLS", "1") != "0"


class SparsePlanBuffers:
    """Device buffers of a ctr_sparse_plan for up to `capacity` slots."""

    def __init__(self, capacity: int, device: torch.device):
        self.capacity = int(capacity)
        self.device = device
        i32 = dict(dtype=torch.int32, device=device)
        c = max(self.capacity, 1)
        self.sorted_slots = torch.empty(c, **i32)
        self.sorted_rows = torch.empty(c, **i32)
        self.pos_seg = torch.empty(c, **i32)
        self.unique_rows = torch.empty(c, **i32)
        self.seg_offsets = torch.empty(c + 1, **i32)
        self.num_unique = torch.zeros(1, **i32)
        self.S = 0
        self._struct = SparsePlan()
        # the plan's own radix scratch (not the per-stream Workspace): plans are built on the
        # plan streams concurrently with steps, and their captured graphs replay there, so
        # their scratch must be private to the plan
        self._ws = None

    def struct(self, rows_are_segments: bool = False) -> SparsePlan:
        """The ctr_sparse_plan of these buffers. rows_are_segments: present each position's
        unique-row ordinal as its row (a table compacted in unique order, row sharding)."""
        s = self._struct
        s.S = self.S
        s.sorted_slots = _p(self.sorted_slots)
        s.sorted_rows = _p(self.pos_seg if rows_are_segments else self.sorted_rows)
        s.pos_seg, s.unique_rows = _p(self.pos_seg), _p(self.unique_rows)
        s.seg_offsets, s.num_unique = _p(self.seg_offsets), _p(self.num_unique)
        return s

    def build(self, idx: torch.Tensor, V: int, err_flag=None) -> "SparsePlanBuffers":
        """idx [B, F] (a batch: the column plan, ctr_sparse_plan_build_cols) or flat ids
        (the LSD plan); both give the same plan bit for bit."""
        F = int(idx.shape[1]) if idx.dim() == 2 and _PLAN_COLS else 0
        idx, it = _idx(idx)
        S = idx.numel()
        if S > self.capacity:
            raise ValueError(f"sparse plan: {S} slots > capacity {self.capacity}")
        self.S = S
        need = lib.ctr_sparse_plan_workspace_bytes(S, int(V))
        if need < 0:
            raise RuntimeError(lib.load().ctr_last_error().decode())
        if self._ws is None or self._ws.numel() < need:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("sparse plan: scratch grown inside a graph capture (build "
                                   "these buffers once eagerly first)")
            full = lib.ctr_sparse_plan_workspace_bytes(max(self.capacity, 1), int(V))
            self._ws = torch.empty(max(need, full, 256), dtype=torch.uint8, device=self.device)
        if F > 0:
            lib.ctr_sparse_plan_build_cols(_p(idx), it, int(V), F, self.struct(), _p(self._ws),
                                           self._ws.numel(), _p(err_flag), _stream())
        else:
            lib.ctr_sparse_plan_build(_p(idx), it, int(V), self.struct(), _p(self._ws),
                                      self._ws.numel(), _p(err_flag), _stream())
        return self

    def build_runs(self, ids: torch.Tensor, n_runs: int, n_rows: int,
                   mask: torch.Tensor) -> "SparsePlanBuffers":
        """The plan of an owner shard's received ids (ctr_sparse_plan_build_runs): n_runs <= 8
        ascending runs of equal length, each row at most once per run, padded with the spare
        row n_rows - 1; bit-identical to build(). mask: int32[ceil(n_rows / 4)] zeros (left
        zero)."""
        _dev(ids, "ids")
        S = ids.numel()
        if ids.dtype != torch.int32 or not ids.is_contiguous() or S % n_runs:
            raise ValueError("build_runs: ids must be contiguous int32, n_runs equal runs")
        if S > self.capacity:
            raise ValueError(f"sparse plan: {S} slots > capacity {self.capacity}")
        if mask.dtype != torch.int32 or mask.numel() < (n_rows + 3) // 4:
            raise ValueError("build_runs: mask must be int32[ceil(n_rows / 4)]")
        self.S = S
        need = lib.ctr_sparse_plan_runs_workspace_bytes(int(n_runs), S // n_runs, int(n_rows))
        if need < 0:
            raise RuntimeError(lib.load().ctr_last_error().decode())
        if self._ws is None or self._ws.numel() < need:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("sparse plan: scratch grown inside a graph capture")
            self._ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        lib.ctr_sparse_plan_build_runs(_p(ids), int(n_runs), S // n_runs, int(n_rows),
                                       self.struct(), _p(mask), _p(self._ws), self._ws.numel(),
                                       _stream())
        return self

    def num_unique_host(self) -> int:
        return int(self.num_unique.item())

    def slot_to_unique(self, out: torch.Tensor | None = None) -> torch.Tensor:
        """int32[S]: the unique-row ordinal of every slot."""
        if out is None:
            out = torch.empty(max(self.capacity, 1), dtype=torch.int32, device=self.device)
        lib.ctr_plan_slot_to_unique(self.struct(), _p(out), _stream())
        return out

    def shard_counts(self, shard_rows: int, n_shards: int, out: torch.Tensor | None = None,
                     max_out: torch.Tensor | None = None) -> torch.Tensor:
        """int64[n_shards]: unique rows owned by each shard (ids // shard_rows); max_out
        (int64[1], n_shards <= 15): their maximum, from the same launch."""
        if out is None:
            out = torch.empty(n_shards, dtype=torch.int64, device=self.device)
        if max_out is not None and (max_out.dtype != torch.int64 or max_out.numel() < 1):
            raise ValueError("shard_counts: max_out must be an int64 tensor")
        lib.ctr_plan_shard_counts_max(self.struct(), int(shard_rows), int(n_shards), _p(out),
                                      _p(max_out), _stream())
        return out


def shard_pack_ids(plan: SparsePlanBuffers, shard_rows: int, V: int, n_shards: int,
                   capacity: int, send: torch.Tensor, counts: torch.Tensor,
                   offsets: torch.Tensor, err_flag: torch.Tensor | None = None,
                   cyclic: bool = False) -> None:
    """The plan's unique rows, per owner shard, into the padded exchange layout
    send[j*capacity + i] (owner-local ids; the owner's spare row past each run); counts /
    offsets: int32[n_shards] (ctr_shard_pack_ids). cyclic: the plan was built over
    shard_permute_ids_ ids (each owner's spare row is then its cyclic row count)."""
    for t, n, k in ((send, "send", n_shards * capacity), (counts, "counts", n_shards),
                    (offsets, "offsets", n_shards)):
        _dev(t, n)
        if t.dtype != torch.int32 or not t.is_contiguous() or t.numel() < k:
            raise ValueError(f"shard_pack_ids: {n} must be contiguous int32 of >= {k}")
    lib.ctr_shard_pack_ids_layout(plan.struct(), int(shard_rows), int(V), int(n_shards),
                                  int(bool(cyclic)), int(capacity), _p(send), _p(counts),
                                  _p(offsets), _p(err_flag), _stream())


def shard_permute_ids_(ids: torch.Tensor, V: int, n_shards: int, shard_rows: int,
                       err_flag: torch.Tensor | None = None) -> torch.Tensor:
    """In place: global row ids r -> (r % n_shards) * shard_rows + r // n_shards, the cyclic
    row-sharding space in which shard j's rows are one block (ctr_shard_permute_ids); ids
    outside [0, V) raise CTR_EFLAG_INDEX in err_flag and map to row 0. int64 or int32."""
    _dev(ids, "ids")
    if ids.dtype not in (torch.int64, torch.int32) or not ids.is_contiguous():
        raise TypeError("shard_permute_ids_: contiguous int64 / int32 ids expected")
    lib.ctr_shard_permute_ids(_p(ids), int(ids.dtype == torch.int64), ids.numel(), int(V),
                              int(n_shards), int(shard_rows), _p(err_flag), _stream())
    return ids


def cu_mask_words(n_cus: int, frac: float) -> list[int]:
    """A CU mask keeping q/8 of n_cus CUs (q = round(8 * frac), 1..8), every XCD its share
    whether the driver numbers CUs XCD by XCD (XCD = c // (n_cus / 8)) or round robin over
    the XCDs (XCD = c % 8): CU c is kept when (c % 8 + c // (n_cus / 8)) % 8 < q (exactly
    balanced when n_cus is a multiple of 64, as MI355X's 256)."""
    q = max(1, min(8, round(8 * frac)))
    per = max(1, n_cus // 8)
    words = [0] * ((n_cus + 31) // 32)
    for c in range(n_cus):
        if (c % 8 + c // per) % 8 < q:
            words[c // 32] |= 1 << (c % 32)
    return words


def cu_masked_stream(words: list[int], device=None) -> torch.cuda.ExternalStream:
    """A torch stream over a HIP stream whose kernels run only on the CUs set in `words`
    (ctr_stream_create_cu_masked). It lives as long as the process."""
    arr = (ctypes.c_uint32 * len(words))(*words)
    out = ctypes.c_void_p()
    lib.ctr_stream_create_cu_masked(ctypes.addressof(arr), len(words), ctypes.addressof(out))
    return torch.cuda.ExternalStream(out.value, device=device)


_STAGE_COPY = os.environ.get("CTR_STAGE_COPY", "1") != "0"  # A/B: the runtime's copies


def batch_stage_copy(ids_dst: torch.Tensor, ids_src: torch.Tensor,
                     y_dst: torch.Tensor | None = None, y_src: torch.Tensor | None = None) -> bool:
    """Copy a batch's ids (and labels) into its input slot in one launch
    (ctr_batch_stage_copy). Only for same-dtype, same-size, contiguous device tensors: returns
    False (nothing launched) otherwise, and the caller copies with torch."""
    if not _STAGE_COPY:
        return False
    pairs = [(ids_dst, ids_src)] + ([(y_dst, y_src)] if y_dst is not None else [])
    for d, s_ in pairs:
        if not (d.is_cuda and s_.is_cuda and d.dtype == s_.dtype and d.numel() == s_.numel()
                and d.is_contiguous() and s_.is_contiguous() and d.device == s_.device):
            return False
    n0 = ids_dst.numel() * ids_dst.element_size()
    n1 = y_dst.numel() * y_dst.element_size() if y_dst is not None else 0
    lib.ctr_batch_stage_copy(_p(ids_dst), _p(ids_src), n0, _p(y_dst) if n1 else None,
                             _p(y_src) if n1 else None, n1, _stream())
    return True


def shard_runs_copy(src: torch.Tensor, dst: torch.Tensor, capacity: int, counts: torch.Tensor,
                    offsets: torch.Tensor, pack: bool) -> torch.Tensor:
    """Rows between the compact order and the padded exchange layout (ctr_shard_runs_copy):
    pack: dst[j*capacity + i] = src[offsets[j] + i] (zeros past counts[j]); else the reverse
    for the runs only."""
    _f32(src, "src")
    _f32(dst, "dst")
    n = counts.numel()
    width = src.shape[1] if src.dim() == 2 else 1
    padded, compact = (dst, src) if pack else (src, dst)
    if padded.shape[0] < n * capacity or (dst.dim() == 2 and dst.shape[1] != width):
        raise ValueError("shard_runs_copy: padded side must hold n_shards * capacity rows")
    lib.ctr_shard_runs_copy(_p(src), _p(dst), int(width), int(capacity), int(n), _p(counts),
                            _p(offsets), int(bool(pack)), _stream())
    return dst


def rows_chunk(capacity: int, K: int, lin: bool) -> int:
    """Floats per (requester, owner) chunk of the rows + linear-weight exchange layout
    (ctr_shard_gather_rows / _rows_pack / _rows_unpack): capacity rows of K floats, then the
    capacity linear weights, padded to a multiple of 4."""
    return capacity * K + ((capacity + 3) // 4 * 4 if lin else 0)


def _rows_lin_check(name, chunked, n_shards, chunk, rows, K, lin):
    _f32(chunked, name)
    if chunked.numel() < n_shards * chunk:
        raise ValueError(f"{name}: needs n_shards * chunk = {n_shards * chunk} floats")
    _f32(rows, "rows")
    if rows.dim() != 2 or rows.shape[1] != K:
        raise ValueError(f"{name}: rows must be [*, {K}]")
    if lin is not None:
        _f32(lin, "lin")


def shard_gather_rows(emb: torch.Tensor, lin: torch.Tensor | None, ids: torch.Tensor,
                      n_shards: int, capacity: int, out: torch.Tensor) -> torch.Tensor:
    """Owner side: the requested rows and their linear weights into the chunked exchange
    layout (ctr_shard_gather_rows); ids int32[n_shards * capacity]."""
    K = emb.shape[1]
    chunk = rows_chunk(capacity, K, lin is not None)
    _rows_lin_check("shard_gather_rows", out, n_shards, chunk, emb, K, lin)
    _dev(ids, "ids")
    if ids.dtype != torch.int32 or ids.numel() < n_shards * capacity:
        raise ValueError("shard_gather_rows: ids must be int32 of n_shards * capacity")
    lib.ctr_shard_gather_rows(_p(emb), _p(lin), K, _p(ids), int(n_shards), int(capacity), chunk,
                              _p(out), _stream())
    return out


def shard_rows_pack(rows: torch.Tensor, lin: torch.Tensor | None, capacity: int,
                    counts: torch.Tensor, offsets: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """Compact rows (+ linear values) -> the chunked exchange layout, zeros past each run
    (ctr_shard_rows_pack)."""
    n, K = counts.numel(), rows.shape[1]
    chunk = rows_chunk(capacity, K, lin is not None)
    _rows_lin_check("shard_rows_pack", out, n, chunk, rows, K, lin)
    lib.ctr_shard_rows_pack(_p(rows), _p(lin), K, int(capacity), chunk, n, _p(counts),
                            _p(offsets), _p(out), _stream())
    return out


def shard_rows_unpack(chunked: torch.Tensor, capacity: int, counts: torch.Tensor,
                      offsets: torch.Tensor, rows: torch.Tensor,
                      lin: torch.Tensor | None = None) -> torch.Tensor:
    """The chunked exchange layout -> compact rows (+ linear values), the runs only
    (ctr_shard_rows_unpack)."""
    n, K = counts.numel(), rows.shape[1]
    chunk = rows_chunk(capacity, K, lin is not None)
    _rows_lin_check("shard_rows_unpack", chunked, n, chunk, rows, K, lin)
    lib.ctr_shard_rows_unpack(_p(chunked), K, int(capacity), chunk, n, _p(counts), _p(offsets),
                              _p(rows), _p(lin), _stream())
    return rows


def ids_add_(ids: torch.Tensor, delta: int) -> torch.Tensor:
    """In place: ids += delta (int32 device ids)."""
    _dev(ids, "ids")
    if ids.dtype != torch.int32 or not ids.is_contiguous():
        raise TypeError("ids_add_: contiguous int32 ids expected")
    lib.ctr_ids_add(_p(ids), ids.numel(), int(delta), _stream())
    return ids


def _seg_ws(plan: SparsePlanBuffers, K: int):
    return Workspace.get(lib.ctr_segment_workspace_bytes(max(plan.S, 1), K), plan.device)


def fm_embedding_grad(plan: SparsePlanBuffers, F: int, emb, gz, sum_e, dx=None, rowmap=None,
                      grad_rows=None, grad_lin=None, compact: bool = False):
    """Per-unique-row gradient sums. compact: `emb` holds the batch's unique rows in plan
    order (row sharding) instead of the whole table."""
    V, K = emb.shape
    cap = max(plan.capacity, 1)
    if grad_rows is None:
        grad_rows = torch.empty(cap, K, dtype=torch.float32, device=emb.device)
    if grad_lin is None:
        grad_lin = torch.empty(cap, dtype=torch.float32, device=emb.device)
    ws = _seg_ws(plan, K)
    lib.ctr_fm_embedding_grad(plan.struct(compact), int(F), int(K), _p(emb), _p(gz), _p(sum_e), _p(dx),
                              _p(grad_rows), _p(grad_lin), _p(rowmap), _p(ws), ws.numel(),
                              _stream())
    return grad_rows, grad_lin


def segment_sum_rows(plan: SparsePlanBuffers, vals, vals_lin=None, rowmap=None, out=None,
                     out_lin=None):
    K = vals.shape[1]
    cap = max(plan.capacity, 1)
    if out is None:
        out = torch.empty(cap, K, dtype=torch.float32, device=vals.device)
    if vals_lin is not None and out_lin is None:
        out_lin = torch.empty(cap, dtype=torch.float32, device=vals.device)
    ws = _seg_ws(plan, K)
    lib.ctr_segment_sum_rows(plan.struct(), int(K), _p(vals), _p(vals_lin), _p(out), _p(out_lin),
                             _p(rowmap), _p(ws), ws.numel(), _stream())
    return out, out_lin


def _deferred_table(emb, m_emb, v_emb, lin, m_lin, v_lin, last):
    from ._lib import DeferredTable
    for t, n in ((emb, "emb"), (m_emb, "m_emb"), (v_emb, "v_emb")):
        _f32(t, n)
    return DeferredTable(_p(emb), _p(m_emb), _p(v_emb), _p(lin), _p(m_lin), _p(v_lin), _p(last))


def shard_row_grads(plan: SparsePlanBuffers, capacity: int, offsets: torch.Tensor,
                    out: torch.Tensor, *, K: int, F: int = 0, emb=None, gz=None, sum_e=None,
                    dx=None, vals=None, lin: bool = False) -> torch.Tensor:
    """A row-sharded requester's per-row gradient sums written straight into the exchange
    chunks (ctr_shard_row_grads; the layout of shard_rows_pack): FM mode (gz: the FM / DeepFM
    slot gradients over the compact table emb) or vals mode (IPNN's per-slot gradients)."""
    _f32(out, "out")
    n = offsets.numel()
    chunk = rows_chunk(capacity, K, lin)
    if out.numel() < n * chunk:
        raise ValueError(f"shard_row_grads: out needs {n * chunk} floats")
    if offsets.dtype != torch.int32:
        raise TypeError("shard_row_grads: offsets must be int32")
    ws = _seg_ws(plan, K)
    lib.ctr_shard_row_grads(plan.struct(gz is not None), int(F), int(K), _p(emb), _p(gz),
                            _p(sum_e), _p(dx), _p(vals), int(bool(lin)), n, _p(offsets),
                            int(capacity), chunk, _p(out), _p(ws), ws.numel(), _stream())
    return out


def fm_embedding_grad_adam(plan: SparsePlanBuffers, F: int, gz, sum_e, dx, table, step_dev,
                           step_table: "AdamStepTable", step: int, betas=(0.9, 0.999), eps=1e-8,
                           weight_decay=0.0, grad_rows=None, grad_lin=None,
                           keep_sums: bool = False) -> None:
    """fm_embedding_grad + adam_deferred_rows(sums, step = *step_dev) with the apply fused
    into the combine pass (ctr_fm_embedding_grad_adam): table = (E, m_E, v_E, w, m_w, v_w,
    last); grad_rows / grad_lin are scratch, holding every row's sum with keep_sums."""
    K = table[0].shape[1]
    ws = _seg_ws(plan, K)
    tab = step_table.ensure(step)
    lib.ctr_fm_embedding_grad_adam(plan.struct(), int(F), int(K), _p(gz), _p(sum_e), _p(dx),
                                   _deferred_table(*table), _p(step_dev), _p(tab),
                                   float(betas[0]), float(betas[1]), float(eps),
                                   float(weight_decay), _p(grad_rows), _p(grad_lin),
                                   int(keep_sums), _p(ws), ws.numel(), _stream())


def segment_sum_rows_adam(plan: SparsePlanBuffers, vals, vals_lin, table, step_dev,
                          step_table: "AdamStepTable", step: int, betas=(0.9, 0.999), eps=1e-8,
                          weight_decay=0.0, out=None, out_lin=None, keep_sums: bool = False) -> None:
    """segment_sum_rows + adam_deferred_rows in one pass (ctr_segment_sum_rows_adam)."""
    K = vals.shape[1]
    ws = _seg_ws(plan, K)
    tab = step_table.ensure(step)
    lib.ctr_segment_sum_rows_adam(plan.struct(), int(K), _p(vals), _p(vals_lin),
                                  _deferred_table(*table), _p(step_dev), _p(tab),
                                  float(betas[0]), float(betas[1]), float(eps),
                                  float(weight_decay), _p(out), _p(out_lin), int(keep_sums),
                                  _p(ws), ws.numel(), _stream())


def rows_to_dense(plan: SparsePlanBuffers, V: int, grad_rows, grad_lin=None):
    K = grad_rows.shape[1]
    dense = torch.zeros(V, K, dtype=torch.float32, device=grad_rows.device)
    dense_lin = (torch.zeros(V, 1, dtype=torch.float32, device=grad_rows.device)
                 if grad_lin is not None else None)
    lib.ctr_rows_to_dense(plan.struct(), int(K), _p(grad_rows), _p(grad_lin), _p(dense),
                          _p(dense_lin), _stream())
    return dense, dense_lin


# --------------------------------------------------------------------------- Adam ----
def adam_scalars(step: int, lr: float, betas=(0.9, 0.999)) -> tuple[float, float]:
    """step_size and sqrt(bias_correction2) exactly as torch/optim/adam.py computes them
    (python doubles)."""
    beta1, beta2 = betas
    bias_correction1 = 1 - beta1 ** step
    bias_correction2 = 1 - beta2 ** step
    return lr / bias_correction1, bias_correction2 ** 0.5


def adam_dense(p, g, m, v, step: int, lr: float, betas=(0.9, 0.999), eps=1e-8,
               weight_decay=0.0, step_dev=None, table=None, planes=None) -> None:
    """One Adam step; with step_dev/table the step index is read on the device (graphs).
    planes: [(offset, Planes)] — sub-matrices p[offset : offset + rows*cols] (row-major,
    the Planes' shape) whose planes are rewritten with the updated values (ctr_adam_dense_planes)."""
    for t, n in ((p, "param"), (g, "grad"), (m, "exp_avg"), (v, "exp_avg_sq")):
        _f32(t, n)
    ss, bc2s = adam_scalars(max(step, 1), lr, betas)
    tab = table.ensure(step) if table is not None else None
    args = (_p(p), _p(g), _p(m), _p(v), p.numel(), ss, bc2s, _p(tab), _p(step_dev),
            float(betas[0]), float(betas[1]), float(eps), float(weight_decay))
    if not planes:
        lib.ctr_adam_dense(*args, _stream())
        return
    views = (PlaneViewDesc * len(planes))(
        *[PlaneViewDesc(int(off), pl.rows, pl.cols, pl.desc) for off, pl in planes])
    lib.ctr_adam_dense_planes(*args, ctypes.cast(views, ctypes.c_void_p), len(planes), _stream())


def adam_embedding(emb, m_emb, v_emb, lin, m_lin, v_lin, rowmap, grad_rows, grad_lin, step: int,
                   lr: float, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, step_dev=None,
                   table=None) -> None:
    V, K = emb.shape
    ss, bc2s = adam_scalars(max(step, 1), lr, betas)
    tab = table.ensure(step) if table is not None else None
    lib.ctr_adam_embedding(_p(emb), _p(m_emb), _p(v_emb), _p(lin), _p(m_lin), _p(v_lin), V, K,
                           _p(rowmap), _p(grad_rows), _p(grad_lin), ss, bc2s, _p(tab),
                           _p(step_dev), float(betas[0]), float(betas[1]), float(eps),
                           float(weight_decay), _stream())


class AdamStepTable:
    """Device table of the per-step Adam scalars for the deferred-exact path:
    tab[2t] = -lr/(1-beta1^t), tab[2t+1] = 1/sqrt(1-beta2^t), computed in python doubles
    exactly like adam_scalars() (so dense and deferred paths see identical fp32 values)."""

    def __init__(self, lr: float, betas, device, capacity: int = 4096):
        self.lr, self.betas, self.device = float(lr), tuple(betas), device
        self.capacity = 0
        self.version = 0  # bumped when the table moves (captured HIP graphs hold its address)
        self.tab = torch.zeros(2, dtype=torch.float32, device=device)
        self.ensure(capacity)

    def _host(self, cap: int) -> torch.Tensor:
        host = torch.zeros(2 * (cap + 1), dtype=torch.float64)
        for t in range(1, cap + 1):
            ss, bc2s = adam_scalars(t, self.lr, self.betas)
            host[2 * t] = -ss
            host[2 * t + 1] = 1.0 / bc2s
        return host.to(torch.float32)

    def ensure(self, step: int) -> torch.Tensor:
        if step > self.capacity:
            cap = max(step, 2 * self.capacity, 1024)
            self.tab = self._host(cap).to(self.device)
            self.capacity = cap
            self.version += 1
        return self.tab

    def set_lr(self, lr: float) -> None:
        """A new learning rate (the driver's `learning_rate += 1e-4` before each epoch's
        Adam): the values are rewritten IN PLACE, so captured HIP graphs, which hold the
        table's address, stay valid and read the new scalars at their next replay."""
        if float(lr) == self.lr:
            return
        self.lr = float(lr)
        self.tab.copy_(self._host(self.capacity), non_blocking=False)


def adam_deferred_rows(emb, m_emb, v_emb, lin, m_lin, v_lin, last, plan: "SparsePlanBuffers",
                       step: int, table: AdamStepTable, betas=(0.9, 0.999), eps=1e-8,
                       weight_decay=0.0, grad_rows=None, grad_lin=None, step_dev=None) -> None:
    """grad_rows None: bring the plan's rows to `step`; else to step-1 and apply `step`.
    step_dev (device int32): read the step there instead (graphs); `step` then only sizes
    the table."""
    V, K = emb.shape
    tab = table.ensure(max(step, 1))
    lib.ctr_adam_deferred_rows(_p(emb), _p(m_emb), _p(v_emb), _p(lin), _p(m_lin), _p(v_lin), V, K,
                               _p(last), plan.struct(), _p(grad_rows), _p(grad_lin),
                               max(int(step), 1), _p(step_dev), _p(tab), float(betas[0]),
                               float(betas[1]), float(eps), float(weight_decay), _stream())


def adam_deferred_entries(emb, m_emb, v_emb, lin, m_lin, v_lin, last, plan: "SparsePlanBuffers",
                          vals: torch.Tensor, vals_lin: torch.Tensor | None, step: int,
                          table: AdamStepTable, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                          skip_row: int = -1, step_dev=None, out=None, out_lin=None,
                          run_len: int = 0) -> None:
    """The owner side of a row-sharded step in one launch (ctr_adam_deferred_entries): each
    unique row of `plan` (over the received entries) stepped with the sequential sum of its
    entries' vals / vals_lin; skip_row left alone. run_len > 0: vals is the chunked exchange
    buffer (shard_rows_pack's layout, rows_chunk(run_len, K, lin) floats per chunk)."""
    V, K = emb.shape
    _f32(vals, "vals")
    chunk = rows_chunk(run_len, K, lin is not None) if run_len else 0
    if run_len == 0 and (vals.dim() != 2 or vals.shape[1] != K):
        raise ValueError(f"adam_deferred_entries: vals must be [entries, {K}]")
    tab = table.ensure(max(step, 1))
    lib.ctr_adam_deferred_entries(_p(emb), _p(m_emb), _p(v_emb), _p(lin), _p(m_lin), _p(v_lin),
                                  V, K, _p(last), plan.struct(), _p(vals), _p(vals_lin),
                                  int(run_len), int(chunk), int(skip_row), max(int(step), 1),
                                  _p(step_dev), _p(tab),
                                  float(betas[0]), float(betas[1]), float(eps),
                                  float(weight_decay), _p(out), _p(out_lin), _stream())


def adam_deferred_catchup_ids(emb, m_emb, v_emb, lin, m_lin, v_lin, last, idx: torch.Tensor,
                              owner: torch.Tensor, step_dev: torch.Tensor, table: AdamStepTable,
                              step_hint: int, betas=(0.9, 0.999), eps=1e-8,
                              weight_decay=0.0) -> None:
    """Bring the rows of a batch's ids to the completed step held in step_dev (device int32),
    no sparse plan needed; owner is an int32[V] scratch. step_hint (>= the device value)
    sizes the step table."""
    V, K = emb.shape
    idx, it = _idx(idx)
    tab = table.ensure(max(step_hint, 1))
    lib.ctr_adam_deferred_catchup_ids(_p(emb), _p(m_emb), _p(v_emb), _p(lin), _p(m_lin), _p(v_lin),
                                      V, K, _p(last), _p(idx), it, idx.numel(), _p(owner),
                                      _p(step_dev), _p(tab), float(betas[0]), float(betas[1]),
                                      float(eps), float(weight_decay), _stream())


def step_begin(step_ctr: torch.Tensor) -> None:
    """ctr[1] = ctr[0] + 1 on the device (int32[2]: completed steps, step in flight)."""
    lib.ctr_step_begin(_p(step_ctr), _stream())


def step_end(step_ctr: torch.Tensor, loss: torch.Tensor | None = None,
             loss_sum: torch.Tensor | None = None) -> None:
    """ctr[0] = ctr[1] on the device; with loss / loss_sum (fp32 [1] / fp64 [1]) also
    loss_sum += loss in double (the driver's epoch loss, no host sync per step)."""
    if loss_sum is None:
        lib.ctr_step_end(_p(step_ctr), _stream())
        return
    _f32(loss, "loss")
    if loss_sum.dtype != torch.float64 or not loss_sum.is_cuda:
        raise TypeError("step_end: loss_sum must be a float64 device tensor")
    lib.ctr_step_end_loss(_p(step_ctr), _p(loss), _p(loss_sum), _stream())


def fm_step_tail(loss_elem: torch.Tensor, gz: torch.Tensor, loss_scale: float,
                 loss_out: torch.Tensor, bias_grad: torch.Tensor, p, g, m, v,
                 table: AdamStepTable, step: int, step_ctr: torch.Tensor, betas=(0.9, 0.999),
                 eps=1e-8, weight_decay=0.0, loss_sum: torch.Tensor | None = None) -> None:
    """The FM step's dense tail in one launch: loss_out = loss_scale * sum(loss_elem),
    bias_grad = sum(gz) (bitwise tensor_sum), the Adam step of the flat dense vector p at
    step ctr[1] (bitwise adam_dense), then step_end(step_ctr) (and loss_sum += loss_out
    in double when given)."""
    if loss_sum is not None and (loss_sum.dtype != torch.float64 or not loss_sum.is_cuda):
        raise TypeError("fm_step_tail: loss_sum must be a float64 device tensor")
    for t, n in ((loss_elem, "loss_elem"), (gz, "gz"), (p, "param"), (g, "grad"),
                 (m, "exp_avg"), (v, "exp_avg_sq")):
        _f32(t, n)
    B = gz.numel()
    if loss_elem.numel() != B or bias_grad.numel() != 1 or loss_out.numel() < 1:
        raise ValueError("fm_step_tail: loss_elem / gz of B elements, one bias gradient")
    if not (g.numel() == m.numel() == v.numel() == p.numel()):
        raise ValueError("fm_step_tail: p, g, m, v of one size")
    tab = table.ensure(step)
    lib.ctr_fm_step_tail(_p(loss_elem), _p(gz), B, float(loss_scale), _p(loss_out),
                         _p(bias_grad), _p(p), _p(g), _p(m), _p(v), p.numel(), _p(tab),
                         _p(step_ctr), float(betas[0]), float(betas[1]), float(eps),
                         float(weight_decay), _p(loss_sum) if loss_sum is not None else None,
                         _stream())


def adam_deferred_flush(emb, m_emb, v_emb, lin, m_lin, v_lin, last, step: int,
                        table: AdamStepTable, betas=(0.9, 0.999), eps=1e-8,
                        weight_decay=0.0) -> None:
    V, K = emb.shape
    tab = table.ensure(step)
    lib.ctr_adam_deferred_flush(_p(emb), _p(m_emb), _p(v_emb), _p(lin), _p(m_lin), _p(v_lin), V, K,
                                _p(last), int(step), _p(tab), float(betas[0]), float(betas[1]),
                                float(eps), float(weight_decay), _stream())


# ------------------------------------------------------------- Feature_Embedding ----
def feature_embedding(idx: torch.Tensor, emb: torch.Tensor, err_flag=None,
                      out_planes: "Planes | None" = None) -> torch.Tensor:
    """Feature_Embedding's state [B, F(F-1)/2 + F*K]; out_planes: also write its three bf16
    planes (the first planes GEMM's A operand)."""
    idx, it = _idx(idx)
    _f32(emb, "feature_embedding.weight")
    B, F = idx.shape
    V, K = emb.shape
    W = F * (F - 1) // 2 + F * K
    out = torch.empty(B, W, dtype=torch.float32, device=emb.device)
    if out_planes is None:
        lib.ctr_feature_embedding_forward(_p(idx), it, B, F, K, V, _p(emb), _p(out),
                                          _p(err_flag), _stream())
        return out
    if out_planes.rows < B or out_planes.cols < W or out_planes.device != emb.device:
        raise ValueError(f"feature_embedding: out_planes must hold [{B}, {W}] on {emb.device}")
    lib.ctr_feature_embedding_forward_planes(_p(idx), it, B, F, K, V, _p(emb), _p(out),
                                             out_planes.desc, _p(err_flag), _stream())
    return out


def ipnn_forward(idx: torch.Tensor, emb: torch.Tensor, out: torch.Tensor | None = None,
                 err_flag=None, planes: "Planes | None" = None) -> torch.Tensor | None:
    """InnerPNN MLP input [B, F*K + F(F-1)/2]: flat embeddings, then the pairwise inner
    products in row-major pair order (p_model.py:187-195). planes: also (or, with
    out=None, only) written as its three bf16 planes — the MLP GEMMs' operand, no split
    pass; returns out (None when only the planes are written)."""
    idx, it = _idx(idx)
    _f32(emb, "feature_embedding.weight")
    B, F = idx.shape
    V, K = emb.shape
    W = F * K + F * (F - 1) // 2
    if out is not None:  # the same checks with or without planes: the C side knows ldc only
        _dev(out, "out")
        if (out.dtype != torch.float32 or out.dim() != 2 or out.shape[0] < B
                or out.shape[1] < W or out.stride(1) != 1):
            raise ValueError(f"ipnn_forward: out must be float32 [>= {B}, >= {W}], unit "
                             "column stride")
    if planes is not None:
        if planes.rows < B or planes.cols < W:
            raise ValueError(f"ipnn_forward: planes [{planes.rows}, {planes.cols}] < [{B}, {W}]")
        lib.ctr_ipnn_forward_planes(_p(idx), it, B, F, K, V, _p(emb), _p(out),
                                    out.stride(0) if out is not None else 0, planes.desc,
                                    _p(err_flag), _stream())
        return out
    if out is None:
        out = torch.empty(B, W, dtype=torch.float32, device=emb.device)
    lib.ctr_ipnn_forward(_p(idx), it, B, F, K, V, _p(emb), _p(out), out.stride(0), _p(err_flag),
                         _stream())
    return out


def ipnn_backward(idx: torch.Tensor, emb: torch.Tensor, dcat: torch.Tensor,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """Per-slot embedding gradients [B*F, K] (slot order) from dL/dcat."""
    idx, it = _idx(idx)
    _f32(emb, "feature_embedding.weight")
    _f32(dcat, "dcat")
    B, F = idx.shape
    V, K = emb.shape
    if dcat.shape[0] < B or dcat.shape[1] < F * K + F * (F - 1) // 2 or dcat.stride(1) != 1:
        raise ValueError("ipnn_backward: dcat must be [B, F*K + F(F-1)/2]")
    if out is None:
        out = torch.empty(B * F, K, dtype=torch.float32, device=emb.device)
    lib.ctr_ipnn_backward(_p(idx), it, B, F, K, V, _p(emb), _p(dcat), dcat.stride(0), _p(out),
                          _stream())
    return out


def ensemble_preds(preds: torch.Tensor, actions: torch.Tensor, prob_weights: torch.Tensor,
                   c_actions: torch.Tensor, labels: torch.Tensor):
    """generate_preds' arithmetic (hybrid_td3_main_per_v10.py:54-164) on [B, M] model pCTRs:
    returns (y_preds [B,1], rewards [B,1], return_c_actions [B,M])."""
    _f32(preds, "preds")
    B, M = preds.shape
    if preds.stride(1) != 1:
        preds = preds.contiguous()
    pw = _f32(prob_weights.reshape(B, M).contiguous(), "prob_weights")
    ca = _f32(c_actions.reshape(B, M).contiguous(), "c_actions")
    act, at = _idx(actions.reshape(B).contiguous(), "actions")
    lab, lt = _idx(labels.reshape(B).contiguous(), "labels")
    dev = preds.device
    y = torch.empty(B, 1, dtype=torch.float32, device=dev)
    r = torch.empty(B, 1, dtype=torch.float32, device=dev)
    rc = torch.empty(B, M, dtype=torch.float32, device=dev)
    rank = torch.empty(max(B, 1), dtype=torch.int32, device=dev)
    lib.ctr_ensemble_preds(_p(preds), B, M, preds.stride(0), _p(act), at, _p(pw), _p(ca),
                           _p(lab), lt, _p(y), _p(r), _p(rc), _p(rank), _stream())
    return y, r, rc


class FFMTables:
    """Device array of the F field tables' data pointers (ctr_ffm_* take `float* const*`);
    rebuilt when a table is re-allocated (Module.to(), load_state_dict into new storage)."""

    def __init__(self):
        self._key = None
        self.ptrs = None

    def get(self, tables) -> torch.Tensor:
        key = tuple(t.data_ptr() for t in tables)
        if key != self._key:
            for t in tables:
                _f32(t, "ffm table")
            self.ptrs = torch.tensor(key, dtype=torch.int64, device=tables[0].device)
            self._key = key
        return self.ptrs


def ffm_forward(idx, tables, ptrs, lin, bias, labels=None, mean_div=None, err_flag=None, out=None):
    """FFM logits z [B] (and with labels: p, per-example loss, dL/dz). out: a dict of this
    function's earlier result for the same B, written in place."""
    idx, it = _idx(idx)
    B, F = idx.shape
    V, K = tables[0].shape
    if len(tables) != F:
        raise ValueError(f"ffm_forward: {len(tables)} tables for {F} fields")
    dev = tables[0].device
    e = lambda: torch.empty(B, dtype=torch.float32, device=dev)  # noqa: E731
    if out is None:
        out = {"z": e()}
        if labels is not None:
            out.update(p=e(), loss_elem=e(), gz=e())
    z = out["z"]
    lib.ctr_ffm_forward(_p(idx), it, B, F, K, V, _p(ptrs), _p(lin), _p(bias), _p(z),
                        _p(labels), float(B if mean_div is None else mean_div), _p(out.get("p")),
                        _p(out.get("loss_elem")), _p(out.get("gz")), _p(err_flag), _stream())
    return out


def ffm_backward(idx, tables, ptrs, gz, keys=None, vals=None):
    """(keys int32 [B*F*(F-1)], vals [B*F*(F-1), K]): every example's table-row gradients
    (into keys / vals when given)."""
    idx, it = _idx(idx)
    B, F = idx.shape
    V, K = tables[0].shape
    n = B * F * (F - 1)
    if keys is None:
        keys = torch.empty(max(n, 1), dtype=torch.int32, device=gz.device)
    if vals is None:
        vals = torch.empty(max(n, 1), K, dtype=torch.float32, device=gz.device)
    if keys.numel() < n or vals.shape[0] < n or vals.shape[1] != K:
        raise ValueError("ffm_backward: keys / vals too small")
    lib.ctr_ffm_backward(_p(idx), it, B, F, K, V, _p(ptrs), _p(_f32(gz.contiguous(), "gz")),
                         _p(keys), _p(vals), _stream())
    return keys[:n], vals[:n]


def ffm_keys(idx, V: int, out=None, err_flag=None) -> torch.Tensor:
    """int32 [B*F*(F-1)]: the (table, row) keys t*V + x of ffm_backward, without values."""
    idx, it = _idx(idx)
    B, F = idx.shape
    n = B * F * (F - 1)
    if out is None:
        out = torch.empty(max(n, 1), dtype=torch.int32, device=idx.device)
    lib.ctr_ffm_keys(_p(idx), it, B, F, int(V), _p(out), _p(err_flag), _stream())
    return out[:n]


# ----------------------------------------------------------------------- REINFORCE ----
def softmax_rows(x: torch.Tensor) -> torch.Tensor:
    _f32(x, "x")
    out = torch.empty_like(x)
    lib.ctr_softmax_rows(_p(x), x.shape[0], x.shape[1], _p(out), _stream())
    return out


def pg_discount_norm(r: torch.Tensor, gamma: float, out32=None):
    """Returns (normalised returns fp64, the same as fp32, stats[mean, std] fp64); out32: a
    float32 [n] tensor to write the fp32 returns into."""
    r = _f32(r.reshape(-1).contiguous(), "rewards")
    n = r.numel()
    out = torch.empty(n, dtype=torch.float64, device=r.device)
    if out32 is None:
        out32 = torch.empty(n, dtype=torch.float32, device=r.device)
    elif (out32.dtype != torch.float32 or out32.numel() != n or not out32.is_contiguous()
          or out32.device != r.device):
        raise ValueError(f"pg_discount_norm: out32 must be a contiguous float32 [{n}] on {r.device}")
    stats = torch.empty(2, dtype=torch.float64, device=r.device)
    lib.ctr_pg_discount_norm(_p(r), n, float(gamma), _p(out), _p(out32), _p(stats), None, 0,
                             _stream())
    return out, out32, stats


def pg_loss_grad(probs: torch.Tensor, acts: torch.Tensor, vt: torch.Tensor, grad_scale=1.0):
    _f32(probs, "probs")
    acts = _dev(acts, "acts").reshape(-1).to(torch.int64).contiguous()
    vt = _f32(vt.reshape(-1).contiguous(), "vt")
    B, A = probs.shape
    loss = torch.empty(1, dtype=torch.float32, device=probs.device)
    dlogits = torch.empty_like(probs)
    lib.ctr_pg_loss_grad(_p(probs), _p(acts), _p(vt), B, A, float(grad_scale), _p(loss),
                         _p(dlogits), None, 0, _stream())
    return loss, dlogits


def pg_vt_mean(vt: torch.Tensor) -> torch.Tensor:
    """Device scalar mean(vt), summed in pg_loss_grad's order."""
    vt = _f32(vt.reshape(-1).contiguous(), "vt")
    out = torch.empty(1, dtype=torch.float32, device=vt.device)
    lib.ctr_pg_vt_mean(_p(vt), vt.numel(), _p(out), _stream())
    return out


def pg_loss_grad_global(probs: torch.Tensor, acts: torch.Tensor, vt_mean: torch.Tensor,
                        grad_scale=1.0):
    """pg_loss_grad for one rank's slice of a data-parallel episode (vt_mean = the
    episode-wide pg_vt_mean); the returned loss is this rank's share of the episode loss."""
    _f32(probs, "probs")
    _f32(vt_mean, "vt_mean")
    acts = _dev(acts, "acts").reshape(-1).to(torch.int64).contiguous()
    B, A = probs.shape
    loss = torch.empty(1, dtype=torch.float32, device=probs.device)
    dlogits = torch.empty_like(probs)
    lib.ctr_pg_loss_grad_global(_p(probs), _p(acts), B, A, _p(vt_mean), float(grad_scale),
                                _p(loss), _p(dlogits), _stream())
    return loss, dlogits
