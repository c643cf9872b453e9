"""ctypes binding of libctr_hip.so (the C ABI declared in include/ctr_hip.h).

This is the only way the package reaches the GPU: there is no CPU or eager-PyTorch
fallback for any op on the hot path. If the library is missing, or was built for
another architecture, every entry point raises instead of computing something else.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(os.environ.get("CTR_HIP_LIB", Path(__file__).resolve().parent / "libctr_hip.so"))

CTR_OK = 0
CTR_IDX_I32, CTR_IDX_I64 = 0, 1
CTR_EFLAG_INDEX = 1
CTR_EFLAG_CAPACITY = 2
EPI_NONE, EPI_BIAS, EPI_BIAS_RELU, EPI_BIAS_RELU_DROP, EPI_GRAD_MASK = range(5)

_vp, _i32, _i64, _f32, _f64, _u64 = C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_double, C.c_uint64


class SparsePlan(C.Structure):
    """Mirror of ``ctr_sparse_plan`` (include/ctr_hip.h)."""
    _fields_ = [("S", _i64), ("sorted_slots", _vp), ("sorted_rows", _vp), ("pos_seg", _vp),
                ("unique_rows", _vp), ("seg_offsets", _vp), ("num_unique", _vp)]


_plan_p = C.POINTER(SparsePlan)


class ColsumJob(C.Structure):
    """Mirror of ``ctr_colsum_job`` (include/ctr_hip.h)."""
    _fields_ = [("X", _vp), ("M", _i64), ("N", _i64), ("ldx", _i64), ("row_w", _vp),
                ("scale", _f32), ("out", _vp)]


_job_p = C.POINTER(ColsumJob)


class PlanesDesc(C.Structure):
    """Mirror of ``ctr_planes`` (include/ctr_hip.h)."""
    _fields_ = [("data", _vp), ("ld", _i64), ("plane_stride", _i64), ("rows", _i64),
                ("cols", _i64)]


_planes_p = C.POINTER(PlanesDesc)


class DeferredTable(C.Structure):
    """Mirror of ``ctr_deferred_table`` (include/ctr_hip.h)."""
    _fields_ = [("emb", _vp), ("m_emb", _vp), ("v_emb", _vp), ("lin", _vp), ("m_lin", _vp),
                ("v_lin", _vp), ("last", _vp)]


_table_p = C.POINTER(DeferredTable)


class PlaneViewDesc(C.Structure):
    """Mirror of ``ctr_plane_view`` (include/ctr_hip.h)."""
    _fields_ = [("offset", _i64), ("rows", _i64), ("cols", _i64), ("planes", PlanesDesc)]


# --- the op-level interface: mirrors of the ctr_<op>_args structs ---------
CTR_OP_FM_FWD, CTR_OP_FM_BWD, CTR_OP_DEEPFM_GATHER_CONCAT, CTR_OP_EMB_SCATTER_ADD = 1, 2, 3, 4
CTR_OP_ADAM_DENSE, CTR_OP_ADAM_ROWWISE, CTR_OP_PAIRWISE_FE, CTR_OP_PG_RETURNS = 5, 6, 7, 8
CTR_OPF_DETERMINISTIC = 1
_IDXF = [("idx", _vp), ("idx_type", _i32), ("B", _i64), ("F", _i32), ("K", _i32), ("V", _i64)]


class FmFwdArgs(C.Structure):
    _fields_ = _IDXF + [("emb", _vp), ("lin", _vp), ("bias", _vp), ("z", _vp), ("sum_e", _vp),
                        ("err_flag", _vp), ("flags", _i32)]


class FmBwdArgs(C.Structure):
    _fields_ = _IDXF + [("emb", _vp), ("sum_e", _vp), ("gz", _vp), ("g_emb", _vp),
                        ("g_lin", _vp), ("g_bias", _vp), ("ws", _vp), ("ws_bytes", _i64),
                        ("err_flag", _vp), ("flags", _i32)]


class DeepfmGatherConcatArgs(C.Structure):
    _fields_ = _IDXF + [("emb", _vp), ("out", _vp), ("err_flag", _vp), ("flags", _i32)]


class EmbScatterAddArgs(C.Structure):
    _fields_ = [("idx", _vp), ("idx_type", _i32), ("n_slots", _i64), ("K", _i32), ("V", _i64),
                ("grad_slots", _vp), ("dense", _vp), ("ws", _vp), ("ws_bytes", _i64),
                ("err_flag", _vp), ("flags", _i32)]


class AdamDenseArgs(C.Structure):
    _fields_ = [("p", _vp), ("g", _vp), ("m", _vp), ("v", _vp), ("n", _i64), ("step", _i64),
                ("lr", _f64), ("beta1", _f64), ("beta2", _f64), ("eps", _f64),
                ("weight_decay", _f64), ("flags", _i32)]


class AdamRowwiseArgs(C.Structure):
    _fields_ = [("emb", _vp), ("m", _vp), ("v", _vp), ("V", _i64), ("K", _i32), ("rows", _vp),
                ("rows_type", _i32), ("n_rows", _i64), ("grad_rows", _vp), ("step", _i64),
                ("lr", _f64), ("beta1", _f64), ("beta2", _f64), ("eps", _f64),
                ("weight_decay", _f64), ("ws", _vp), ("ws_bytes", _i64), ("err_flag", _vp),
                ("flags", _i32)]


class PairwiseFeArgs(C.Structure):
    _fields_ = _IDXF + [("emb", _vp), ("out", _vp), ("err_flag", _vp), ("flags", _i32)]


class PgReturnsArgs(C.Structure):
    _fields_ = [("r", _vp), ("n", _i64), ("gamma", _f64), ("vt", _vp), ("vt_f32", _vp),
                ("ws", _vp), ("ws_bytes", _i64), ("flags", _i32)]


OP_ARGS = {"fm_fwd": FmFwdArgs, "fm_bwd": FmBwdArgs, "deepfm_gather_concat": DeepfmGatherConcatArgs,
           "emb_scatter_add": EmbScatterAddArgs, "adam_dense": AdamDenseArgs,
           "adam_rowwise": AdamRowwiseArgs, "pairwise_fe": PairwiseFeArgs,
           "pg_returns": PgReturnsArgs}


# name -> (restype, argtypes); the list is the whole ABI and tests/test_abi.py checks it
# against the header.
SIGNATURES = {
    "ctr_abi_version": (_i32, []),
    "ctr_last_error": (C.c_char_p, []),
    "ctr_device_count": (_i32, []),
    "ctr_embedding_gather": (_i32, [_vp, _i64, _i32, _vp, _i32, _i64, _vp, _vp, _vp]),
    "ctr_fm_forward": (_i32, [_vp, _i32, _i64, _i32, _i32, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                              _vp, _f32, _vp, _vp, _vp, _vp, _vp]),
    "ctr_bce_sigmoid": (_i32, [_vp, _vp, _i64, _f32, _vp, _vp, _vp, _vp]),
    "ctr_deepfm_head": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _f32, _f32, _vp, _vp, _vp,
                               _vp, _vp, _vp]),
    "ctr_gemm_f32_workspace_bytes": (_i64, [_i32, _i32, _i64, _i64, _i64]),
    "ctr_gemm_f32": (_i32, [_i32, _i32, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i32,
                            _vp, _vp, _i64, _f32, _f32, _u64, _u64, _vp, _vp, _i64, _vp]),
    "ctr_gemm_f32_ex_workspace_bytes": (_i64, [_i32, _i32, _i32, _i64, _i64, _i64]),
    "ctr_gemm_f32_ex": (_i32, [_i32, _i32, _i32, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp,
                               _i64, _i32, _vp, _vp, _i64, _f32, _f32, _u64, _u64, _vp, _vp,
                               _i64, _vp]),
    "ctr_gemm_resolved_algo": (_i32, [_i32]),
    "ctr_split_planes": (_i32, [_vp, _i64, _i64, _i64, _planes_p, _vp]),
    "ctr_gemm_planes_workspace_bytes": (_i64, [_i32, _i32, _i64, _i64, _i64]),
    "ctr_gemm_planes": (_i32, [_i32, _i32, _i64, _i64, _i64, _planes_p, _planes_p, _vp, _i64,
                               _planes_p, _i32, _vp, _vp, _i64, _f32, _f32, _u64, _u64, _vp, _vp,
                               _i64, _vp]),
    "ctr_gemm_planes_lastcol": (_i32, [_i32, _i32, _i64, _i64, _i64, _planes_p, _planes_p, _vp,
                                       _i64, _planes_p, _i32, _vp, _vp, _i64, _f32, _f32, _u64,
                                       _u64, _vp, _vp, _vp, _i64, _vp]),
    "ctr_gemm_planes_config": (_i32, [_i32, _i32, _i64, _i64, _i64, _vp, _vp, _vp, _vp]),
    "ctr_fm_forward_planes": (_i32, [_vp, _i32, _i64, _i32, _i32, _i64, _vp, _vp, _vp, _vp, _vp,
                                     _planes_p, _vp, _vp]),
    "ctr_deepfm_head_planes": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _f32, _f32, _vp, _vp,
                                      _vp, _vp, _vp, _planes_p, _vp]),
    "ctr_reduce_workspace_bytes": (_i64, [_i64, _i64]),
    "ctr_sum_f32": (_i32, [_vp, _i64, _f32, _vp, _vp, _i64, _vp]),
    "ctr_colsum_f32": (_i32, [_vp, _i64, _i64, _i64, _vp, _f32, _vp, _vp, _i64, _vp]),
    "ctr_colsum_multi_workspace_bytes": (_i64, [_i32, _job_p]),
    "ctr_colsum_multi_f32": (_i32, [_i32, _job_p, _vp, _i64, _vp]),
    "ctr_transpose_f32": (_i32, [_vp, _i64, _i64, _i64, _vp, _i64, _vp]),
    "ctr_sparse_plan_workspace_bytes": (_i64, [_i64, _i64]),
    "ctr_sparse_plan_build": (_i32, [_vp, _i32, _i64, _plan_p, _vp, _i64, _vp, _vp]),
    "ctr_sparse_plan_build_cols": (_i32, [_vp, _i32, _i64, _i64, _plan_p, _vp, _i64, _vp, _vp]),
    "ctr_plan_slot_to_unique": (_i32, [_plan_p, _vp, _vp]),
    "ctr_plan_shard_counts": (_i32, [_plan_p, _i64, _i32, _vp, _vp]),
    "ctr_plan_shard_counts_max": (_i32, [_plan_p, _i64, _i32, _vp, _vp, _vp]),
    "ctr_adam_deferred_entries": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _plan_p,
                                         _vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _f64, _f64,
                                         _f64, _f64, _vp, _vp, _vp]),
    "ctr_shard_row_grads": (_i32, [_plan_p, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _vp,
                                   _i64, _i64, _vp, _vp, _i64, _vp]),
    "ctr_shard_gather_rows": (_i32, [_vp, _vp, _i32, _vp, _i32, _i64, _i64, _vp, _vp]),
    "ctr_shard_rows_pack": (_i32, [_vp, _vp, _i32, _i64, _i64, _i32, _vp, _vp, _vp, _vp]),
    "ctr_shard_rows_unpack": (_i32, [_vp, _i32, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp]),
    "ctr_ids_add": (_i32, [_vp, _i64, _i32, _vp]),
    "ctr_shard_pack_ids": (_i32, [_plan_p, _i64, _i64, _i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "ctr_shard_pack_ids_layout": (_i32, [_plan_p, _i64, _i64, _i32, _i32, _i64, _vp, _vp, _vp,
                                         _vp, _vp]),
    "ctr_shard_permute_ids": (_i32, [_vp, _i32, _i64, _i64, _i32, _i64, _vp, _vp]),
    "ctr_stream_create_cu_masked": (_i32, [_vp, _i32, _vp]),
    "ctr_stream_destroy": (_i32, [_vp]),
    "ctr_shard_runs_copy": (_i32, [_vp, _vp, _i64, _i64, _i32, _vp, _vp, _i32, _vp]),
    "ctr_batch_stage_copy": (_i32, [_vp, _vp, _i64, _vp, _vp, _i64, _vp]),
    "ctr_sparse_plan_runs_workspace_bytes": (_i64, [_i32, _i64, _i64]),
    "ctr_sparse_plan_build_runs": (_i32, [_vp, _i32, _i64, _i64, _plan_p, _vp, _vp, _i64, _vp]),
    "ctr_segment_workspace_bytes": (_i64, [_i64, _i32]),
    "ctr_fm_embedding_grad": (_i32, [_plan_p, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                     _vp, _i64, _vp]),
    "ctr_segment_sum_rows": (_i32, [_plan_p, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "ctr_rows_to_dense": (_i32, [_plan_p, _i32, _vp, _vp, _vp, _vp, _vp]),
    "ctr_adam_dense": (_i32, [_vp, _vp, _vp, _vp, _i64, _f64, _f64, _vp, _vp, _f64, _f64, _f64,
                              _f64, _vp]),
    "ctr_fm_embedding_grad_adam": (_i32, [_plan_p, _i32, _i32, _vp, _vp, _vp, _table_p, _vp, _vp,
                                          _f64, _f64, _f64, _f64, _vp, _vp, _i32, _vp, _i64, _vp]),
    "ctr_segment_sum_rows_adam": (_i32, [_plan_p, _i32, _vp, _vp, _table_p, _vp, _vp, _f64, _f64,
                                         _f64, _f64, _vp, _vp, _i32, _vp, _i64, _vp]),
    "ctr_adam_dense_planes": (_i32, [_vp, _vp, _vp, _vp, _i64, _f64, _f64, _vp, _vp, _f64, _f64,
                                     _f64, _f64, _vp, _i32, _vp]),
    "ctr_adam_embedding": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _f64,
                                  _f64, _vp, _vp, _f64, _f64, _f64, _f64, _vp]),
    "ctr_adam_deferred_rows": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _plan_p, _vp,
                                      _vp, _i64, _vp, _vp, _f64, _f64, _f64, _f64, _vp]),
    "ctr_adam_deferred_catchup_ids": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp,
                                             _i32, _i64, _vp, _vp, _vp, _f64, _f64, _f64, _f64,
                                             _vp]),
    "ctr_step_begin": (_i32, [_vp, _vp]),
    "ctr_step_end": (_i32, [_vp, _vp]),
    "ctr_step_end_loss": (_i32, [_vp, _vp, _vp, _vp]),
    "ctr_fm_step_tail": (_i32, [_vp, _vp, _i64, _f32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                                _vp, _f64, _f64, _f64, _f64, _vp, _vp]),
    "ctr_adam_deferred_flush": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _vp,
                                       _f64, _f64, _f64, _f64, _vp]),
    "ctr_feature_embedding_forward": (_i32, [_vp, _i32, _i64, _i32, _i32, _i64, _vp, _vp, _vp,
                                             _vp]),
    "ctr_feature_embedding_forward_planes": (_i32, [_vp, _i32, _i64, _i32, _i32, _i64, _vp,
                                                    _vp, _planes_p, _vp, _vp]),
    "ctr_ensemble_preds": (_i32, [_vp, _i64, _i32, _i64, _vp, _i32, _vp, _vp, _vp, _i32, _vp, _vp,
                                  _vp, _vp, _vp]),
    "ctr_ffm_forward": (_i32, [_vp, _i32, _i64, _i32, _i32, _i64, _vp, _vp, _vp, _vp, _vp, _f32,
                               _vp, _vp, _vp, _vp, _vp]),
    "ctr_ffm_keys": (_i32, [_vp, _i32, _i64, _i32, _i64, _vp, _vp, _vp]),
    "ctr_ffm_backward": (_i32, [_vp, _i32, _i64, _i32, _i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "ctr_csv_to_bin": (_i32, [C.c_char_p, C.c_char_p, _vp, _vp, _vp]),
    "ctr_bin_info": (_i32, [C.c_char_p, _vp, _vp, _vp, _vp]),
    "ctr_ipnn_forward": (_i32, [_vp, _i32, _i64, _i32, _i32, _i64, _vp, _vp, _i64, _vp, _vp]),
    "ctr_ipnn_forward_planes": (_i32, [_vp, _i32, _i64, _i32, _i32, _i64, _vp, _vp, _i64,
                                       _planes_p, _vp, _vp]),
    "ctr_ipnn_backward": (_i32, [_vp, _i32, _i64, _i32, _i32, _i64, _vp, _vp, _i64, _vp, _vp]),
    "ctr_softmax_rows": (_i32, [_vp, _i64, _i32, _vp, _vp]),
    "ctr_pg_workspace_bytes": (_i64, [_i64]),
    "ctr_pg_discount_norm": (_i32, [_vp, _i64, _f64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "ctr_pg_loss_grad": (_i32, [_vp, _vp, _vp, _i64, _i32, _f32, _vp, _vp, _vp, _i64, _vp]),
    "ctr_pg_vt_mean": (_i32, [_vp, _i64, _vp, _vp]),
    "ctr_pg_loss_grad_global": (_i32, [_vp, _vp, _i64, _i32, _vp, _f32, _vp, _vp, _vp]),
    "ctr_workspace_bytes": (_i64, [_i32, C.POINTER(_i64), _i32]),
    **{f"ctr_op_{op}": (_i32, [C.POINTER(st), _vp]) for op, st in OP_ARGS.items()},
}


class CtrHipError(RuntimeError):
    pass


class _Lib:
    """Lazily loaded handle; attribute access returns a checked wrapper."""

    def __init__(self) -> None:
        self._dll = None

    def load(self) -> C.CDLL:
        if self._dll is None:
            if not LIB_PATH.exists():
                raise CtrHipError(
                    f"{LIB_PATH} not found: build it with `python -m rl_ctr_prediction_amd.build_lib` "
                    "(hipcc, gfx950). There is no CPU fallback for the HIP hot path.")
            dll = C.CDLL(str(LIB_PATH))
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(dll, name)
                fn.restype = res
                fn.argtypes = args
            self._dll = dll
        return self._dll

    def raw(self, name: str):
        return getattr(self.load(), name)

    def __getattr__(self, name: str):
        if not name.startswith("ctr_"):
            raise AttributeError(name)
        fn = self.raw(name)
        res = SIGNATURES[name][0]
        if res is not _i32 or name in ("ctr_abi_version", "ctr_device_count"):
            self.__dict__[name] = fn
            return fn

        def checked(*args):
            rc = fn(*args)
            if rc != CTR_OK:
                msg = self.load().ctr_last_error().decode(errors="replace")
                raise CtrHipError(f"{name} failed (status {rc}): {msg}")
            return rc

        checked.__name__ = name
        self.__dict__[name] = checked  # later lookups skip __getattr__ (host cost per call)
        return checked


lib = _Lib()


def exported_symbols() -> list[str]:
    """Names of every C-ABI entry point (used by the CPU test of the library)."""
    return list(SIGNATURES)
