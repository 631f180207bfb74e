"""ctypes binding of libkgat_hip.so (the C-ABI declared in include/kgat_hip.h).

The library is built in-tree (``make -C csrc``, or ``__graft_entry__.build()``)
and loaded after ``torch`` so that it binds to the HIP runtime torch already
loaded (both carry the soname libamdhip64.so.7).  There is no fallback: if the
library is missing every op raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (must be loaded first: shares its HIP runtime)

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("KGAT_HIP_LIB", _HERE / "libkgat_hip.so"))

KGAT_MAX_TABLES = 8

c_i32, c_i64, c_f32, c_u64, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p


class CSR(ctypes.Structure):
    """Mirror of ``kgat_csr``."""

    _fields_ = [
        ("rowptr", c_vp), ("col", c_vp), ("val", c_vp), ("n_rows", c_i64), ("nnz", c_i64),
        ("long_rows", c_vp), ("long_seg_off", c_vp), ("seg_row", c_vp), ("seg_beg", c_vp),
        ("n_long", c_i32), ("n_seg", c_i32), ("seg_len", c_i32), ("long_threshold", c_i32),
        ("seg_order", c_vp),
    ]


class AdamTensor(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("n", ctypes.c_int64), ("step_size", ctypes.c_float), ("bc2_sqrt", ctypes.c_float)]


KGAT_ADAM_MAX_TENSORS = 16
KGAT_COMM_ID_BYTES = 128


class Tables(ctypes.Structure):
    """Mirror of ``kgat_tables``."""

    _fields_ = [("ptr", c_vp * KGAT_MAX_TABLES), ("ld", c_i64 * KGAT_MAX_TABLES),
                ("width", c_i32 * KGAT_MAX_TABLES), ("count", c_i32)]


KGAT_IDS_MAX = 4
KGAT_HOP_PRECLEARED = 1


class Ids(ctypes.Structure):
    """Mirror of ``kgat_ids``."""

    _fields_ = [("ptr", c_vp * KGAT_IDS_MAX), ("n", c_i64 * KGAT_IDS_MAX), ("count", c_i32)]


KGAT_NFM_MAX_LAYERS = 4


class NFMNet(ctypes.Structure):
    """Mirror of ``kgat_nfm``."""

    _fields_ = [("V", c_vp), ("ld_v", c_i64), ("w_lin", c_vp), ("b_lin", c_vp), ("W", c_vp * KGAT_NFM_MAX_LAYERS),
                ("b", c_vp * KGAT_NFM_MAX_LAYERS), ("dims", c_i32 * (KGAT_NFM_MAX_LAYERS + 1)), ("n_layers", c_i32),
                ("W_out", c_vp), ("dropout_p", c_f32), ("seed", c_u64)]


# name -> (restype, argtypes)
_SIGNATURES = {
    "kgat_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "kgat_version": (ctypes.c_int, []),
    "kgat_csr_plan": (ctypes.c_int, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "kgat_csr_plan_cols": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp,
                                          c_vp, c_vp]),
    "kgat_csr_seg_order": (ctypes.c_int, [c_vp, c_vp, c_i32, c_vp]),
    "kgat_spmm_csr_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_vp, c_i64,
                                         c_vp]),
    "kgat_biinter_fwd_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                            c_i32, c_i32, c_f32, c_u64, c_vp, c_vp, c_vp]),
    "kgat_biinter_fwd_rows_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                                 c_i64, c_i32, c_i32, c_f32, c_u64, c_vp, c_vp, c_vp]),
    "kgat_biinter_bwd_workspace": (c_i64, [c_i64, c_i32, c_i32]),
    "kgat_spmm_csr_masked_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64,
                                                c_i32, c_vp, c_i64, c_vp]),
    "kgat_spmm_csr_masked_ex_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp,
                                                   c_i64, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "kgat_spmm_csr_masked_adam_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp,
                                                     c_vp, c_vp, c_i64, c_i32, c_f32, c_f32, c_f32, c_f32, c_f32, c_vp,
                                                     c_i64, c_vp]),
    "kgat_spmm_csr_masked_adam_ex_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_i64, c_vp, c_i64, c_vp,
                                                        c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_f32, c_f32, c_f32,
                                                        c_f32, c_vp, c_vp, c_i64, c_vp]),
    "kgat_map_rank": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp]),
    "kgat_map_bits": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp]),
    "kgat_hop_compact_work_bytes": (c_i64, [c_i64]),
    "kgat_hop_compact": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "kgat_biinter_bwd_hop_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp,
                                                c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                c_i64, c_i64, c_i32, c_i32, c_i32, c_f32, c_vp, c_i64, c_vp]),
    "kgat_biinter_bwd_hop_ex_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                                                   c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                   c_vp, c_i64, c_i64, c_i32, c_i32, c_i32, c_f32, c_vp, c_i64, c_vp,
                                                   c_vp, c_vp, c_i64, c_vp]),
    "kgat_frontier_hop_work_bytes": (c_i64, [c_i64]),
    "kgat_frontier_hop_ex": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            c_vp, c_vp, c_i64, c_i32, c_vp]),
    "kgat_frontier_hop": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                         c_vp, c_i64, c_vp]),
    "kgat_rows_union": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                                       c_vp]),
    "kgat_rows_merge_f32": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i32, c_vp, c_i64, c_i32, c_vp, c_vp, c_i64, c_vp,
                                           c_i64, c_f32, c_vp]),
    "kgat_spmm_csr_masked_rows_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp,
                                                     c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp]),
    "kgat_spmm_csr_masked_rows_ex_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_vp, c_i64, c_vp, c_i64,
                                                        c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i32,
                                                        c_vp, c_i64, c_vp]),
    "kgat_spmm_csr_rows_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32,
                                              c_vp, c_i64, c_vp]),
    "kgat_biinter_fwd_tiles_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                                  c_vp, c_i32, c_i32, c_f32, c_u64, c_vp, c_vp, c_vp]),
    "kgat_biinter_fwd_list_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                                 c_vp, c_vp, c_i64, c_i32, c_i32, c_f32, c_u64, c_vp, c_vp, c_vp]),
    "kgat_biinter_bwd_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                                            c_vp, c_vp, c_vp, c_vp, c_vp,
                                            c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_f32,
                                            c_u64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "kgat_bpr_fwd_f32": (ctypes.c_int, [ctypes.POINTER(Tables), c_vp, c_vp, c_vp, c_i32, c_f32, c_vp, c_vp, c_vp]),
    "kgat_bpr_bwd_f32": (ctypes.c_int, [ctypes.POINTER(Tables), c_i32, c_vp, c_vp, c_vp, c_i32, c_f32, c_vp, c_vp,
                                        c_vp, c_i64, c_vp, c_vp]),
    "kgat_bpr_fwd_ex_f32": (ctypes.c_int, [ctypes.POINTER(Tables), c_vp, c_vp, c_vp, c_i32, c_f32, c_vp, c_vp, c_vp,
                                           c_vp]),
    "kgat_bpr_bwd_multi_f32": (ctypes.c_int, [ctypes.POINTER(Tables), c_i32, c_vp, c_vp, c_vp, c_i32, c_f32, c_vp,
                                              c_vp, ctypes.POINTER(Tables), c_vp, c_vp, c_vp]),
    "kgat_cf_begin": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                     c_i64, c_vp]),
    "kgat_cf_begin_ex": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                        c_vp, c_i64, ctypes.POINTER(CSR), c_vp, c_vp, c_i32, c_vp]),
    "kgat_row_softmax_work_floats": (c_i64, [ctypes.POINTER(CSR)]),
    "kgat_row_softmax_plan_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_vp, c_i64, c_vp]),
    "kgat_frontier_build": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "kgat_frontier_reset": (ctypes.c_int, [c_vp, c_i32, c_vp, c_vp]),
    "kgat_transr_work_floats": (c_i64, [c_i32, c_i32, c_i32]),
    "kgat_transr_fwd_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_f32,
                                           c_vp, c_vp, c_vp]),
    "kgat_transr_fwd_ex_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp,
                                              c_i32, c_f32, c_vp, c_vp, c_vp]),
    "kgat_transr_bwd_workspace_floats": (c_i64, [c_i32, c_i32, c_i32, c_i32]),
    "kgat_transr_bwd_ex_f32": (ctypes.c_int, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp,
                                              c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "kgat_adam_rows_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_i64, c_f32, c_f32, c_f32,
                                          c_f32, c_f32, c_vp, c_vp]),
    "kgat_transr_bwd_f32": (ctypes.c_int, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp,
                                           c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "kgat_edge_logits_f32": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                            c_vp, c_vp, c_vp, c_vp, c_i32, c_f32, c_u64, c_vp, c_vp, c_vp]),
    "kgat_slot_sum_f32": (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "kgat_row_softmax_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp]),
    "kgat_row_softmax_ex_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp]),
    "kgat_biinter_gemm_state_floats": (c_i64, [c_i64, c_i32, c_i32]),
    "kgat_biinter_gemm_work_floats": (c_i64, [c_i64, c_i32, c_i32]),
    "kgat_biinter_fwd_gemm_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                                 c_i32, c_i32, c_f32, c_u64, c_vp, c_vp, c_i64, c_vp]),
    "kgat_biinter_bwd_gemm_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp,
                                                 c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32,
                                                 c_i32, c_f32, c_u64, c_vp, c_vp, c_i64, c_vp]),
    "kgat_biinter_gemm_bits_work_floats": (c_i64, [c_i64, c_i32, c_i32]),
    "kgat_biinter_bwd_gemm_bits_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                                                      c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                                      c_i64, c_i32, c_i32, c_f32, c_vp, c_vp, c_i64, c_vp]),
    "kgat_sample_cf_batch": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_i32, c_u64, c_u64, c_vp, c_vp, c_vp]),
    "kgat_nfm_batch_work_bytes": (c_i64, [c_i64]),
    "kgat_nfm_batch_rowptr": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "kgat_nfm_batch_fill": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                           c_vp]),
    "kgat_sample_kg_batch": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_i32, c_u64, c_u64, c_vp, c_vp, c_vp,
                                            c_vp]),
    "kgat_adam_multi_f32": (ctypes.c_int, [ctypes.POINTER(AdamTensor), c_i32, c_f32, c_f32, c_f32, c_vp]),
    "kgat_adam_multi_ex_f32": (ctypes.c_int, [ctypes.POINTER(AdamTensor), c_i32, c_f32, c_f32, c_f32, c_vp, c_vp]),
    "kgat_spmm_csr_masked_adam_multi_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_i64, c_vp, c_i64, c_vp,
                                                           c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_f32, c_f32, c_f32,
                                                           c_f32, c_vp, c_vp, c_i64, ctypes.POINTER(AdamTensor), c_i32,
                                                           c_vp]),
    "kgat_edge_logits_gemm_work_floats": (c_i64, [c_i64, c_i32]),
    "kgat_edge_logits_gemm_f32": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                 c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i32, c_f32, c_u64, c_vp, c_vp,
                                                 c_vp, c_i64, c_vp]),
    "kgat_gather_rows_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp]),
    "kgat_scatter_rows_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_vp]),
    "kgat_add_f32": (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp]),
    "kgat_mask_rows_f32": (ctypes.c_int, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_f32, c_vp]),
    "kgat_topk_f32": (ctypes.c_int, [c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp]),
    "kgat_rank_metrics_f32": (ctypes.c_int, [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "kgat_score_f32": (ctypes.c_int, [ctypes.POINTER(Tables), c_vp, c_i32, c_vp, c_i32, c_vp, c_i64, c_vp]),
    "kgat_coo_rowptr": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp]),
    "kgat_nfm_act_floats": (c_i64, [ctypes.POINTER(NFMNet), c_i64]),
    "kgat_nfm_fwd_f32": (ctypes.c_int, [ctypes.POINTER(NFMNet), c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "kgat_nfm_loss_f32": (ctypes.c_int, [ctypes.POINTER(NFMNet), c_vp, c_i32, c_f32, c_vp, c_vp, c_vp]),
    "kgat_nfm_bwd_workspace": (c_i64, [ctypes.POINTER(NFMNet), c_i64, c_i64]),
    "kgat_nfm_bwd_f32": (ctypes.c_int, [ctypes.POINTER(NFMNet), c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_f32,
                                        c_vp, c_i64, c_vp, c_vp, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_vp, c_vp,
                                        c_i64, c_vp]),
    "kgat_adam_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32, c_vp]),
    "kgat_gather_f32": (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "kgat_fill_f32": (ctypes.c_int, [c_vp, c_i64, c_f32, c_vp]),
    "kgat_map_build": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp]),
    "kgat_map_build_checked": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "kgat_ids_sanitize_i32": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "kgat_map_compose": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i32, c_vp, c_vp]),
    "kgat_adam_lazy_catchup_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp, c_i32, c_vp,
                                                  c_vp, c_vp, c_i32, c_f32, c_f32, c_f32, c_vp]),
    "kgat_adam_lazy_rows_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp,
                                               c_vp, c_vp, c_i32, c_f32, c_f32, c_f32, c_f32, c_f32, c_vp, c_vp]),
    "kgat_adam_multi_sched_f32": (ctypes.c_int, [ctypes.POINTER(AdamTensor), c_i32, c_f32, c_f32, c_f32, c_vp, c_vp,
                                                 c_vp, c_vp, c_i32, c_vp, c_vp]),
    "kgat_adam_lazy_catchup_sched_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp,
                                                        c_vp, c_vp, c_i32, c_f32, c_f32, c_f32, c_vp]),
    "kgat_adam_lazy_rows_sched_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp,
                                                     c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_f32, c_f32, c_f32, c_vp,
                                                     c_vp, c_i32, c_vp, c_vp]),
    "kgat_spmm_csr_masked_adam_block_f32": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_vp, c_i64, c_vp, c_i64, c_i64,
                                                           c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_f32, c_f32,
                                                           c_f32, c_f32, c_vp, c_vp, c_i64, c_vp]),
    "kgat_csr_mark_rows": (ctypes.c_int, [ctypes.POINTER(CSR), c_vp, c_i64, c_i64, c_vp, c_vp]),
    "kgat_biinter_gemm_rows_work_floats": (c_i64, [c_i64, c_i32, c_i32]),
    "kgat_biinter_bwd_gemm_rows_work_floats": (c_i64, [c_i64, c_i32, c_i32]),
    "kgat_biinter_bwd_gemm_rows_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                                      c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp,
                                                      c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_f32, c_u64, c_vp,
                                                      c_i64, c_vp]),
    "kgat_biinter_bwd_gemm_rows_ex_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                                      c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp,
                                                      c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_f32, c_u64, c_vp,
                                                      c_i64, c_i32, c_vp]),
    "kgat_biinter_fwd_gemm_rows_f32": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                                      c_vp, c_i64, c_i64, c_i32, c_i32, c_f32, c_u64, c_vp, c_vp,
                                                      c_i64, c_vp]),
    "kgat_ids_check": (ctypes.c_int, [ctypes.POINTER(Ids), c_i64, c_vp, c_vp, c_vp]),
    "kgat_ids_check_ex": (ctypes.c_int, [ctypes.POINTER(Ids), c_i64, c_vp, c_vp, c_vp, c_vp]),
    "kgat_ids_check_multi": (ctypes.c_int, [ctypes.POINTER(Ids), ctypes.POINTER(c_i64), c_vp, c_vp, c_vp, c_vp]),
    "kgat_gemm_f32": (ctypes.c_int, [c_i32, c_i32, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp,
                                     c_i64, c_i64, c_i64, c_i32, c_vp]),
    "kgat_comm_load": (ctypes.c_int, [ctypes.c_char_p]),
    "kgat_comm_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "kgat_comm_unique_id": (ctypes.c_int, [c_vp]),
    "kgat_comm_init": (ctypes.c_int, [c_i32, c_i32, c_vp, c_i32, ctypes.POINTER(c_vp)]),
    "kgat_comm_destroy": (ctypes.c_int, [c_vp]),
    "kgat_comm_rank": (ctypes.c_int, [c_vp, ctypes.POINTER(c_i32), ctypes.POINTER(c_i32)]),
    "kgat_comm_allreduce_sum_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp]),
    "kgat_comm_allgather_rows": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp]),
    "kgat_comm_reduce_scatter_rows_f32": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp]),
    "kgat_comm_ring_exchange": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp]),
    "kgat_comm_allgatherv": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.POINTER(c_i64), c_vp]),
    "kgat_comm_gather_at": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), c_vp]),
    "kgat_comm_alltoallv": (ctypes.c_int, [c_vp, c_vp, ctypes.POINTER(c_i64), c_vp, ctypes.POINTER(c_i64), c_vp]),
    "kgat_synth_open": (ctypes.c_int, [c_i64, c_i64, c_u64, ctypes.c_double, ctypes.c_int, ctypes.POINTER(c_vp)]),
    "kgat_synth_close": (None, [c_vp]),
    "kgat_synth_info": (ctypes.c_int, [c_vp, c_vp]),
    "kgat_synth_row_offsets": (ctypes.c_int, [c_vp, c_vp]),
    "kgat_synth_triples": (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "kgat_synth_shard_build": (ctypes.c_int, [c_vp, c_i64, c_i64, ctypes.POINTER(c_i64)]),
    "kgat_synth_shard_build_ex": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i32, ctypes.POINTER(c_i64)]),
    "kgat_synth_shard_copy": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp]),
}

_lib = None


def exported_symbols() -> list[str]:
    return sorted(_SIGNATURES)


def lib() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raise if it is not built."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"KGAT HIP library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        handle = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = lib().kgat_strerror(status).decode()
        raise RuntimeError(f"{what} failed: {msg} (status {status})")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)
