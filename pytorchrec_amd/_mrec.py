"""ctypes binding of libmrec.so (the C ABI declared in include/mrec.h).

The library is built in-tree (``pytorchrec_amd/lib/libmrec.so``, see
``pytorchrec_amd/build.py``).  There is deliberately no fallback: any op that
runs on a GPU tensor goes through this library, and if the library is missing
the call raises ``MrecUnavailable`` instead of silently running something else.

``torch`` must be imported before the library is loaded so that the HIP runtime
torch ships (SONAME libamdhip64.so.7) is the one libmrec binds to — one runtime
per process, shared streams and device pointers.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.environ.get("MREC_LIB_PATH") or os.path.join(LIB_DIR, "libmrec.so")

ABI_VERSION = 29
MAX_TABLES = 64
BWD_MAX_BATCH = 8192
BWD_HASH_MAX_BATCH = 4096  # batches up to this use the hash plan (fusable into a GEMM launch)

# mrec_status
OK, EINVAL, EOOB, EHIP, ERCCL, ENOSPC = range(6)
# mrec_dtype
F32, BF16, I32, I64 = 0, 1, 2, 3
# interact flags
INTERACT_FM2 = 1
INTERACT_FIRST_ORDER = 2
# bwd modes
BWD_DENSE_GRAD, BWD_SGD, BWD_SGD_SR = 0, 1, 2
BWD_ADAGRAD, BWD_ROWWISE_ADAGRAD, BWD_ADAM = 3, 4, 5  # fused optimizers (bank.optim)
OPT_DECOUPLED_WD, OPT_NO_BIAS_CORRECTION = 1, 2

_STATUS_NAMES = {OK: "MREC_OK", EINVAL: "MREC_EINVAL", EOOB: "MREC_EOOB", EHIP: "MREC_EHIP",
                 ERCCL: "MREC_ERCCL", ENOSPC: "MREC_ENOSPC"}


class MrecUnavailable(RuntimeError):
    """libmrec.so is missing or unloadable: the HIP path cannot run."""


class MrecError(RuntimeError):
    def __init__(self, fn, status, msg):
        super().__init__(f"{fn} failed: {_STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class TableBank(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p),
                ("row_offset", ctypes.POINTER(ctypes.c_int64)),
                ("rows", ctypes.POINTER(ctypes.c_int64)),
                ("n_tables", ctypes.c_int32),
                ("dim", ctypes.c_int32),
                ("row_stride", ctypes.c_int32),
                ("has_w", ctypes.c_int32),
                ("dtype", ctypes.c_int),
                ("optim", ctypes.c_void_p)]


class Optim(ctypes.Structure):
    """mrec_optim: fused row-sparse optimizer state (include/mrec.h)."""
    _fields_ = [("kind", ctypes.c_int32), ("lr", ctypes.c_float),
                ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_float), ("weight_decay", ctypes.c_float),
                ("grad_scale", ctypes.c_float),
                ("flags", ctypes.c_int32),
                ("state0", ctypes.c_void_p), ("state1", ctypes.c_void_p),
                ("row_step", ctypes.c_void_p), ("d_t", ctypes.c_void_p),
                ("state_ld", ctypes.c_int64)]


class Ids(ctypes.Structure):
    _fields_ = [("field_ptr", ctypes.POINTER(ctypes.c_void_p)),
                ("dtype", ctypes.c_int),
                ("stride", ctypes.c_int64),
                ("chunk", ctypes.c_int64),
                ("chunk_stride", ctypes.c_int64),
                ("pad_negative", ctypes.c_int32)]


class Operand(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("dtype", ctypes.c_int), ("layout", ctypes.c_int),
                ("ld", ctypes.c_int64)]


class Epilogue(ctypes.Structure):
    _fields_ = [("bias", ctypes.c_void_p), ("act", ctypes.c_int32),
                ("mul", ctypes.c_void_p), ("ld_mul", ctypes.c_int64),
                ("add", ctypes.c_void_p), ("ld_add", ctypes.c_int64),
                ("aux", ctypes.c_void_p), ("ld_aux", ctypes.c_int64),
                ("mask", ctypes.c_void_p), ("ld_mask", ctypes.c_int64),
                ("ones_out", ctypes.c_void_p),
                ("update", ctypes.c_int32), ("lr", ctypes.c_float),
                ("img_row", ctypes.c_void_p), ("ld_img_row", ctypes.c_int64),
                ("img_tr", ctypes.c_void_p), ("ld_img_tr", ctypes.c_int64),
                ("img_kind", ctypes.c_int32)]


IMG_ROW_TR, IMG_TOWER = 0, 1


class GemmCall(ctypes.Structure):
    _fields_ = [("M", ctypes.c_int64), ("N", ctypes.c_int64), ("K", ctypes.c_int64),
                ("A", ctypes.POINTER(Operand)), ("B", ctypes.POINTER(Operand)),
                ("b_ones_col", ctypes.c_int64), ("b_cols", ctypes.c_int64),
                ("epi", ctypes.POINTER(Epilogue)), ("C", ctypes.c_void_p), ("c_dtype", ctypes.c_int),
                ("ldc", ctypes.c_int64), ("split_k", ctypes.c_int32),
                ("workspace", ctypes.c_void_p), ("ws_bytes", ctypes.c_size_t),
                ("phase", ctypes.c_int32)]


GEMM_FULL, GEMM_PARTIAL, GEMM_REDUCE = 0, 1, 2


class PlanJob(ctypes.Structure):
    _fields_ = [("bank", ctypes.POINTER(TableBank)), ("ids", ctypes.POINTER(Ids)),
                ("batch", ctypes.c_int64), ("workspace", ctypes.c_void_p),
                ("ws_bytes", ctypes.c_size_t), ("d_oob_flag", ctypes.c_void_p),
                ("d_step", ctypes.c_void_p)]


class GivenGrads(ctypes.Structure):
    """mrec_given_grads (include/mrec.h)."""
    _fields_ = [("g_occ", ctypes.c_void_p), ("g_ld", ctypes.c_int64), ("chunk", ctypes.c_int64),
                ("chunk_stride", ctypes.c_int64), ("wire", ctypes.c_void_p),
                ("rec_bytes", ctypes.c_int32), ("wire_dtype", ctypes.c_int),
                ("pref", ctypes.c_void_p), ("cap_rows", ctypes.c_int32)]


class GradRecords(ctypes.Structure):
    """mrec_grad_records (include/mrec.h, ABI 26)."""
    _fields_ = [("wire", ctypes.c_void_p), ("rec_bytes", ctypes.c_int32), ("pref", ctypes.c_void_p),
                ("cap", ctypes.c_int32), ("cap_rows", ctypes.c_int32)]


class WireRows(ctypes.Structure):
    """mrec_wire_rows (include/mrec.h, ABI 28)."""
    _fields_ = [("wire", ctypes.c_void_p), ("rec_bytes", ctypes.c_int32), ("hdr", ctypes.c_void_p),
                ("parts", ctypes.c_int32), ("cap", ctypes.c_int32), ("cap_rows", ctypes.c_int32),
                ("pref", ctypes.c_void_p), ("d_overflow", ctypes.c_void_p)]


class HeadFinishJob(ctypes.Structure):
    _fields_ = [("part", ctypes.c_void_p), ("ldp", ctypes.c_int64), ("batch", ctypes.c_int64),
                ("H", ctypes.c_int32), ("ns", ctypes.c_int32), ("g", ctypes.c_void_p),
                ("update", ctypes.c_int32), ("lr", ctypes.c_float), ("w", ctypes.c_void_p),
                ("bias", ctypes.c_void_p), ("ws", ctypes.c_void_p), ("b2", ctypes.c_void_p),
                ("dw_out", ctypes.c_void_p), ("db_out", ctypes.c_void_p),
                ("dws_out", ctypes.c_void_p), ("db2_out", ctypes.c_void_p)]

class SgdJob(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("g", ctypes.c_void_p), ("N", ctypes.c_int64),
                ("K", ctypes.c_int64), ("ldw", ctypes.c_int64), ("ldg", ctypes.c_int64),
                ("lr", ctypes.c_float), ("img_row", ctypes.c_void_p), ("ld_row", ctypes.c_int64),
                ("img_tr", ctypes.c_void_p), ("ld_tr", ctypes.c_int64),
                ("img_kind", ctypes.c_int32)]


TOWER_BCE, TOWER_FORWARD, TOWER_GIVEN_DZ = 0, 1, 2  # mrec_tower_args.mode


class TowerArgs(ctypes.Structure):
    """mrec_tower_args (include/mrec.h)."""
    _fields_ = [("batch", ctypes.c_int64), ("n_layers", ctypes.c_int32),
                ("width", ctypes.c_int32 * 5),
                ("x0", ctypes.c_void_p), ("ld_x0", ctypes.c_int64),
                ("w_fwd", ctypes.c_void_p * 4), ("w_bwd", ctypes.c_void_p * 4),
                ("bias", ctypes.c_void_p * 4),
                ("head_w", ctypes.c_void_p), ("head_b", ctypes.c_void_p),
                ("base", ctypes.c_void_p), ("xs", ctypes.c_void_p), ("ld_xs", ctypes.c_int64),
                ("ns", ctypes.c_int32), ("ws", ctypes.c_void_p), ("b2", ctypes.c_void_p),
                ("y", ctypes.c_void_p),
                ("h_out", ctypes.c_void_p * 4), ("ld_h", ctypes.c_int64 * 4),
                ("dh_out", ctypes.c_void_p * 4), ("ld_dh", ctypes.c_int64 * 4),
                ("dx0", ctypes.c_void_p), ("ld_dx0", ctypes.c_int64),
                ("z", ctypes.c_void_p), ("dz", ctypes.c_void_p),
                ("part", ctypes.c_void_p), ("ldp", ctypes.c_int64),
                ("loss_part", ctypes.c_void_p), ("ticket", ctypes.c_void_p),
                ("loss", ctypes.c_void_p), ("kfrag", ctypes.c_int32), ("x0_img", ctypes.c_void_p),
                ("mode", ctypes.c_int32), ("dz_in", ctypes.c_void_p),
                ("n_cross", ctypes.c_int32), ("cross_w_fwd", ctypes.c_void_p * 3),
                ("cross_w_bwd", ctypes.c_void_p * 3), ("cross_bias", ctypes.c_void_p * 3),
                ("cross_x_img", ctypes.c_void_p * 3), ("cross_dz_img", ctypes.c_void_p * 3)]


class TowerDwArgs(ctypes.Structure):
    """mrec_tower_dw_args (include/mrec.h)."""
    _fields_ = [("n_layers", ctypes.c_int32), ("batch", ctypes.c_int64),
                ("n_out", ctypes.c_int32 * 8), ("n_in", ctypes.c_int32 * 8),
                ("dy_img", ctypes.c_void_p * 8), ("x_img", ctypes.c_void_p * 8),
                ("ws", ctypes.c_void_p * 8), ("ldws", ctypes.c_int64 * 8),
                ("splits", ctypes.c_int32)]


class FeedJob(ctypes.Structure):
    """mrec_feed_job (include/mrec.h, ABI 27; widen_bytes ABI 29)."""
    _fields_ = [("dst", ctypes.c_void_p), ("host_base", ctypes.c_void_p),
                ("record_bytes", ctypes.c_int64), ("n_records", ctypes.c_int64),
                ("d_state", ctypes.c_void_p), ("widen_bytes", ctypes.c_int64)]


LAYOUT_ROW, LAYOUT_COL = 0, 1
ACT_NONE, ACT_RELU = 0, 1

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_fp = ctypes.POINTER(ctypes.c_float)
_bank_p = ctypes.POINTER(TableBank)
_ids_p = ctypes.POINTER(Ids)
_op_p = ctypes.POINTER(Operand)
_epi_p = ctypes.POINTER(Epilogue)

# name -> (restype, argtypes); the set the header declares (checked by tests)
SIGNATURES = {
    "mrec_abi_version": (ctypes.c_int, []),
    "mrec_emb_optim_state_ld": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    "mrec_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "mrec_comm_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.POINTER(ctypes.c_void_p)]),
    "mrec_comm_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "mrec_comm_world": (ctypes.c_int32, [ctypes.c_void_p]),
    "mrec_comm_rank": (ctypes.c_int32, [ctypes.c_void_p]),
    "mrec_a2a_ids": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int64, ctypes.c_void_p]),
    "mrec_a2a_rows_fwd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_int64, ctypes.c_void_p]),
    "mrec_a2a_rows_bwd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_int64, ctypes.c_void_p]),
    "mrec_allreduce_sum_f32": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                              ctypes.c_void_p]),
    "mrec_emb_optim_flush": (ctypes.c_int, [_bank_p, ctypes.c_int, ctypes.c_float,
                                            ctypes.c_void_p]),
    "mrec_last_error": (ctypes.c_char_p, []),
    "mrec_emb_gather_fwd": (ctypes.c_int, [_bank_p, _ids_p, _i64, _vp, ctypes.c_int, _i64, _vp,
                                           _vp, _vp]),
    "mrec_interact_fwd": (ctypes.c_int, [_bank_p, _ids_p, _i64, _vp, _i32, _i64, _vp, _vp, _i32,
                                         _vp, ctypes.c_int, _i64, _i32, _vp, _vp, _vp, _vp]),
    "mrec_interact_fwd_ex": (ctypes.c_int, [_bank_p, _ids_p, _i64, _vp, _i32, _i64, _vp, _vp, _i32,
                                            _vp, ctypes.c_int, _i64, _i32, _vp, _vp, _vp,
                                            ctypes.POINTER(PlanJob), _vp]),
    "mrec_interact_fwd_rec": (ctypes.c_int, [_bank_p, _ids_p, _i64, _vp, _i32, _i64, _vp, _vp, _i32,
                                             _vp, ctypes.c_int, _i64, _i32, _vp, _vp, _vp,
                                             ctypes.POINTER(PlanJob), ctypes.POINTER(WireRows), _vp]),
    "mrec_fm2_fwd": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp]),
    "mrec_fm2_bwd": (ctypes.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _vp]),
    "mrec_emb_bwd_workspace_size": (ctypes.c_size_t, [_i32, _i64]),
    "mrec_emb_bwd_plan": (ctypes.c_int, [_bank_p, _ids_p, _i64, _vp, ctypes.c_size_t, _vp, _vp,
                                         _vp]),
    "mrec_emb_bwd_apply": (ctypes.c_int, [_bank_p, _i64, _vp, ctypes.c_size_t, _vp, ctypes.c_int,
                                          _i64, _vp, _vp, _vp, ctypes.c_int, _i64, _vp,
                                          ctypes.c_int, _f32, ctypes.c_uint64, _vp, _vp, _vp]),
    "mrec_emb_bwd_apply_ex": (ctypes.c_int, [_bank_p, _i64, _vp, ctypes.c_size_t, _vp, ctypes.c_int,
                                             _i64, _vp, _vp, _vp, ctypes.c_int, _i64, _vp,
                                             ctypes.c_int, _f32, ctypes.c_uint64, _vp, _vp, _i32,
                                             ctypes.POINTER(GemmCall), _vp]),
    "mrec_emb_bwd_apply_given": (ctypes.c_int, [_bank_p, _i64, _vp, ctypes.c_size_t, _vp,
                                                ctypes.c_int, _i64, _vp, _vp, _vp, ctypes.c_int,
                                                _i64, _vp, _vp, _i64, _i64, _i64, ctypes.c_int,
                                                _f32, ctypes.c_uint64, _vp, _vp, _i32,
                                                ctypes.POINTER(GemmCall), _vp]),
    "mrec_emb_bwd_apply_rec": (ctypes.c_int, [_bank_p, _i64, _vp, ctypes.c_size_t, _vp,
                                              ctypes.c_int, _i64, _vp, _vp, _vp, ctypes.c_int,
                                              _i64, _vp, ctypes.POINTER(GradRecords), _i32,
                                              ctypes.POINTER(GemmCall), _vp]),
    "mrec_emb_bwd_apply_wire": (ctypes.c_int, [_bank_p, _i64, _vp, ctypes.c_size_t, _vp, _i32, _i32,
                                               _vp, _i32, _i64, _i64, ctypes.c_int, _f32,
                                               ctypes.c_uint64, _vp, _vp, _i32,
                                               ctypes.POINTER(GemmCall), _vp]),
    "mrec_emb_bwd_apply_wire_sgd": (ctypes.c_int, [_bank_p, _i64, _vp, ctypes.c_size_t, _vp, _i32,
                                                   _i32, _vp, _i32, _i64, _i64, ctypes.c_int, _f32,
                                                   ctypes.c_uint64, _vp, _vp, _i32,
                                                   ctypes.POINTER(GemmCall), _vp, _i32, _vp]),
    "mrec_shard_bucketize": (ctypes.c_int, [_ids_p, _i32, ctypes.POINTER(ctypes.c_int64), _i64,
                                            _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "mrec_shard_gather": (ctypes.c_int, [_bank_p, _vp, _i32, _i32, _vp, _vp]),
    "mrec_shard_lookup_grad": (ctypes.c_int, [_i64, _i32, _i32, _i32, _vp, _vp, ctypes.c_int,
                                              _i64, _vp, _vp, _vp, ctypes.c_int, _i64, _vp, _vp,
                                              _i64, _vp]),
    "mrec_gemm_workspace_size": (ctypes.c_size_t, [_i64, _i64, _i64, _i32]),
    "mrec_gemm": (ctypes.c_int, [_i64, _i64, _i64, _op_p, _op_p, _i64, _i64, _epi_p,
                                 _vp, ctypes.c_int, _i64, _i32, _vp, ctypes.c_size_t, _vp]),
    "mrec_gemm_multi": (ctypes.c_int, [_i32, ctypes.POINTER(GemmCall), _vp]),
    "mrec_tower_dw": (ctypes.c_int, [ctypes.POINTER(TowerDwArgs), ctypes.POINTER(HeadFinishJob), _vp]),
    "mrec_tower_dw_ex": (ctypes.c_int, [ctypes.POINTER(TowerDwArgs), ctypes.POINTER(HeadFinishJob),
                                        ctypes.POINTER(FeedJob), _vp]),
    "mrec_kfrag_elems": (_i64, [_i64, _i64]),
    "mrec_kfrag_pack": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _vp]),
    "mrec_gemm_multi_ex": (ctypes.c_int, [_i32, ctypes.POINTER(GemmCall), ctypes.POINTER(PlanJob),
                                          ctypes.POINTER(HeadFinishJob), _vp]),
    "mrec_weight_prep": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "mrec_sgd_multi": (ctypes.c_int, [_i32, ctypes.POINTER(SgdJob), _vp]),
    "mrec_sgd_table_bytes": (ctypes.c_size_t, []),
    "mrec_sgd_table_build": (ctypes.c_int, [_i32, ctypes.POINTER(SgdJob), _vp, ctypes.c_size_t,
                                            ctypes.POINTER(ctypes.c_int32)]),
    "mrec_batch_stage": (ctypes.c_int, [_vp, _vp, _i64, _vp]),
    "mrec_batch_stage_cursor": (ctypes.c_int, [_vp, _vp, _i64, _i64, _vp, _vp]),
    "mrec_batch_stage_ex": (ctypes.c_int, [_vp, _vp, _i64, _i64, _vp]),
    "mrec_batch_stage_job": (ctypes.c_int, [ctypes.POINTER(FeedJob), _vp]),
    "mrec_dcn_cross_bwd_prep": (ctypes.c_int, [_i64, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp,
                                               _i64, _vp, _i64, _i32, _vp, _i64, _vp]),
    "mrec_emb_bwd_large_workspace_size": (ctypes.c_size_t, [_bank_p, _i64]),
    "mrec_emb_bwd_large_zero_bytes": (ctypes.c_size_t, [_bank_p, _i64]),
    "mrec_emb_bwd_large_error_offset": (ctypes.c_size_t, []),
    "mrec_kernel_clock": (None, [_vp, _i32]),
    "mrec_kernel_clock_used": (_i32, []),
    "mrec_emb_bwd_large_plan": (ctypes.c_int, [_bank_p, _ids_p, _i64, _vp, ctypes.c_size_t, _vp,
                                               _vp]),
    "mrec_emb_bwd_large_apply": (ctypes.c_int, [_bank_p, _i64, _vp, ctypes.c_size_t, _vp,
                                                ctypes.c_int, _i64, _vp, _vp, _vp, ctypes.c_int,
                                                _i64, _vp, ctypes.c_int, _f32, ctypes.c_uint64,
                                                _vp, _vp, _vp]),
    "mrec_emb_bwd_large_fused": (ctypes.c_int, [_bank_p, _ids_p, _i64, _vp, ctypes.c_size_t, _vp,
                                                _vp, ctypes.c_int, _i64, _vp, _vp, _vp,
                                                ctypes.c_int, _i64, _vp, ctypes.c_int, _f32,
                                                ctypes.c_uint64, _vp, _vp, _vp]),
    "mrec_emb_bwd_large_fused_given": (ctypes.c_int, [_bank_p, _ids_p, _i64, _vp, ctypes.c_size_t,
                                                      _vp, ctypes.POINTER(GivenGrads), ctypes.c_int,
                                                      _f32, ctypes.c_uint64, _vp, _vp, _i32,
                                                      ctypes.POINTER(GemmCall), _vp]),
    "mrec_emb_bwd_large_fused_ex": (ctypes.c_int, [_bank_p, _ids_p, _i64, _vp, ctypes.c_size_t,
                                                   _vp, _vp, ctypes.c_int, _i64, _vp, _vp, _vp,
                                                   ctypes.c_int, _i64, _vp, ctypes.c_int, _f32,
                                                   ctypes.c_uint64, _vp, _vp, _i32,
                                                   ctypes.POINTER(GemmCall), _vp]),
    "mrec_head_fwd": (ctypes.c_int, [_vp, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp]),
    "mrec_head_bwd": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp, _i64, _vp, _i64, _vp]),
    "mrec_bce_fwd": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "mrec_bce_bwd": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "mrec_din_feat_fwd": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _i64, _vp]),
    "mrec_din_pool_fwd": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32,
                                         _i32, _vp, _vp, _i64, _vp]),
    "mrec_din_pool_bwd": (ctypes.c_int, [_vp, _i64, _vp, _vp, _i64, _i64, _i32, _i32, _vp, _vp,
                                         _i64, _vp]),
    "mrec_din_feat_bwd": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32,
                                         _i32, _vp, _i64, _vp, _i64, _vp]),
    "mrec_din_feat_bwd_rows": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i64, _i32,
                                              _i32, _vp, _i64, _vp, _i64, _vp]),
    "mrec_din_lookup_ids": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _i64, _i32, _i64, _i32, _vp,
                                           _vp, _vp]),
    "mrec_din_gather": (ctypes.c_int, [_bank_p, _vp, _vp, _vp, _i64, _vp, _i64, _i32, _i64, _i32,
                                        _vp, _vp, _vp, _i32, _i64, _vp, _vp]),
    "mrec_din_att_supported": (ctypes.c_int32, [_i32, _i32, _i32]),
    "mrec_din_att_parts": (ctypes.c_int64, [_i64]),
    "mrec_din_att_param_count": (ctypes.c_int64, [_i32, _i32, _i32]),
    "mrec_din_att_fwd": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _i64, _vp,
                                        _i32, _vp, _i64, _vp, _i32, _vp, _vp, _vp, _vp, _i64,
                                        _vp]),
    "mrec_din_att_bwd": (ctypes.c_int, [_vp, _i64, _i64, _i32, _i32, _vp, _i64, _vp, _i32, _vp,
                                        _i64, _vp, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp,
                                        _i64, _vp]),
    "mrec_din_att_wgrad": (ctypes.c_int, [_vp, _i64, _i32, _i32, _i32, _vp, _f32, _vp, _i64, _vp,
                                          _vp, _i64, _vp, _vp, _vp, _vp]),
    "mrec_ctr_head_parts": (ctypes.c_int64, [_i64]),
    "mrec_ctr_head_fwd": (ctypes.c_int, [_vp, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64,
                                         _i32, _vp, _vp, _i32, _vp, _vp, _vp, _i64, _vp, _i64,
                                         _vp, _vp, _vp, _vp]),
    "mrec_ctr_head_finish": (ctypes.c_int, [_vp, _i64, _i64, _i32, _i32, _vp, _i32, _f32, _vp, _vp,
                                            _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mrec_colsum": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _i64, _i64, _i64, _vp, _vp, _i32,
                                   _f32, _vp]),
    "mrec_shard_bucketize_dedup": (ctypes.c_int, [_ids_p, _i32, ctypes.POINTER(ctypes.c_int64),
                                                  _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "mrec_shard_bucketize_dedup_ex": (ctypes.c_int, [_ids_p, _i32, ctypes.POINTER(ctypes.c_int64),
                                                     _i64, _i32, _i32, _i64, _vp, _vp, _vp, _vp,
                                                     _vp]),
    "mrec_shard_dedup_scratch_bytes": (ctypes.c_size_t, [_i32, _i64, _i32, _i32]),
    "mrec_shard_bucketize_dedup_q": (ctypes.c_int, [_ids_p, _i32, ctypes.POINTER(ctypes.c_int64),
                                                    _i64, _i32, _i32, _i64, _i32, _vp,
                                                    ctypes.c_size_t, _vp, _vp, _vp, _vp, _vp]),
    "mrec_shard_wire_bytes": (_i32, [_i32, _i32, _i32]),
    "mrec_shard_gather_wire": (ctypes.c_int, [_bank_p, _vp, _i32, _i32, _i32, _vp, _vp,
                                              ctypes.POINTER(PlanJob), _vp]),
    "mrec_shard_gather_wire_ex": (ctypes.c_int, [_bank_p, _vp, _i32, _i32, _i32, _vp, _vp, _vp,
                                                 ctypes.POINTER(PlanJob), _vp]),
    "mrec_shard_wire_unpack": (ctypes.c_int, [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _i64,
                                              _i32, _vp, _i64, _vp, _vp]),
    "mrec_shard_wire_unpack_ex": (ctypes.c_int, [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp,
                                                 _i64, _i32, _vp, _i64, _vp, _vp, _vp]),
    "mrec_shard_wire_pack": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp,
                                            _vp]),
    "mrec_tower_fwd_bwd": (ctypes.c_int, [ctypes.POINTER(TowerArgs), _vp]),
    "mrec_tower_image_elems": (ctypes.c_int64, [_i64, _i64, _i32]),
    "mrec_tower_weight_prep": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp]),
}

_lib = None
_lock = threading.Lock()


def lib():
    """Load (once) and return the ctypes handle; raise MrecUnavailable if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise MrecUnavailable(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
        try:
            handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise MrecUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        v = handle.mrec_abi_version()
        # (MREC_ABI_ANY=1: an older diagnostic build for an A/B timing, tools/gpu_ab.sh)
        if v != ABI_VERSION and os.environ.get("MREC_ABI_ANY") != "1":
            raise MrecUnavailable(f"libmrec ABI {v} != expected {ABI_VERSION}; rebuild it")
        _lib = handle
        return _lib


def available() -> bool:
    try:
        lib()
        return True
    except MrecUnavailable:
        return False


def check(fn_name: str, status: int):
    if status != OK:
        msg = lib().mrec_last_error()
        raise MrecError(fn_name, status, msg.decode() if msg else "")


def call(fn_name: str, *args):
    check(fn_name, getattr(lib(), fn_name)(*args))


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(t: torch.dtype) -> int:
    if t == torch.float32:
        return F32
    if t == torch.bfloat16:
        return BF16
    if t == torch.int32:
        return I32
    if t == torch.int64:
        return I64
    raise TypeError(f"unsupported dtype for libmrec: {t}")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


class BankDesc:
    """Keeps the ctypes TableBank and its host arrays alive."""

    def __init__(self, weight: torch.Tensor, row_offset, rows, dim: int, has_w: bool):
        n = len(rows)
        if n > MAX_TABLES:
            raise ValueError(f"at most {MAX_TABLES} tables per bank")
        self._off = (ctypes.c_int64 * n)(*[int(x) for x in row_offset])
        self._rows = (ctypes.c_int64 * n)(*[int(x) for x in rows])
        self.weight = weight
        self.struct = TableBank(weight.data_ptr(), self._off, self._rows, n, int(dim),
                                int(weight.shape[1]), int(bool(has_w)), dtype_code(weight.dtype),
                                None)
        self.optim = None  # Optim struct kept alive with its state tensors (set_optim)

    def set_optim(self, optim: "Optim | None"):
        self.optim = optim
        self.struct.optim = ctypes.cast(ctypes.pointer(optim), ctypes.c_void_p) if optim else None

    def ref(self):
        self.struct.data = self.weight.data_ptr()
        return ctypes.byref(self.struct)


class IdsDesc:
    """Per-field id tensors (each [B] contiguous, or columns of a [B, F] tensor)."""

    def __init__(self, fields, stacked: torch.Tensor | None = None, chunk: int = 0,
                 chunk_stride: int = 0, pad_negative: bool = False):
        if stacked is not None:
            n = stacked.shape[1]
            base = stacked.data_ptr()
            es = stacked.element_size()
            self.tensors = [stacked]
            ptrs = [base + f * es for f in range(n)]
            stride = stacked.stride(0)
            dt = stacked.dtype
            if stacked.stride(1) != 1:
                raise ValueError("stacked ids must be contiguous along fields")
        else:
            self.tensors = list(fields)
            n = len(self.tensors)
            dt = self.tensors[0].dtype
            for t in self.tensors:
                if t.dtype != dt or t.dim() != 1 or (t.numel() > 1 and t.stride(0) != 1):
                    raise ValueError("per-field ids must be 1-D contiguous tensors of one dtype")
            ptrs = [t.data_ptr() for t in self.tensors]
            stride = 1
        self._ptrs = (ctypes.c_void_p * n)(*ptrs)
        self.struct = Ids(ctypes.cast(self._ptrs, ctypes.POINTER(ctypes.c_void_p)),
                          dtype_code(dt), int(stride), int(chunk), int(chunk_stride),
                          int(bool(pad_negative)))

    @classmethod
    def exchange_view(cls, buf: torch.Tensor, n_tables: int, cap: int, part: int = 0):
        """Owner-side view of a receive buffer of W parts [n_tables][cap] (int32, -1 =
        pad; ``part`` = int32 per part when the parts carry more, e.g. the compact
        exchange's counts header): table f's W*cap entries at
        buf[f*cap + (i // cap) * part + i % cap]."""
        flat = buf.reshape(-1)
        d = cls([flat[f * cap:] for f in range(n_tables)], chunk=cap,
                chunk_stride=part or n_tables * cap, pad_negative=True)
        return d

    def ref(self):
        return ctypes.byref(self.struct)
