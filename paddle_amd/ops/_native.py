"""ctypes binding of the gfx950 kernel library (``lib/libpaddle_amd_kernels.so``).

Every launcher has a flat C ABI: raw device pointers, sizes, scalars and the
``hipStream_t`` of torch's *current* stream, so launches are ordered with the
rest of the step and are capturable into HIP graphs.

Policy (mirrors the reference's CPU-kernel / CUDA-kernel split):
GPU tensors ALWAYS go through these kernels -- if the library is missing on a
machine with a GPU we raise instead of silently falling back; CPU tensors use the
PyTorch reference implementations in :mod:`paddle_amd.ops.reference`.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from .. import _build

_lock = threading.Lock()
_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float
_LP = ctypes.POINTER(ctypes.c_long)

_SIGS = {
    "pa_norm_fwd": [_I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _F, _P],
    "pa_norm_bwd": [_I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P],
    "pa_rope": [_I, _I, _P, _L, _P, _L, _P, _P, _P, _L, _L, _I, _I, _I, _I, _P],
    "pa_swiglu_fwd": [_I, _P, _P, _L, _I, _P],
    "pa_gelu_fwd": [_I, _P, _P, _L, _P],
    "pa_bias_grad_blocks": [_L, _I],
    "pa_bias_act_bwd": [_I, _I, _P, _P, _P, _P, _P, _L, _I, _P],
    "pa_swiglu_bwd": [_I, _P, _P, _P, _L, _I, _P],
    "pa_embedding_fwd": [_I, _P, _P, _P, _L, _I, _L, _P],
    "pa_embedding_bwd": [_I, _P, _P, _P, _L, _I, _L, _P],
    "pa_cast": [_I, _I, _P, _P, _L, _P],
    "pa_act_fwd": [_I, _I, _P, _P, _L, _F, _F, _P],
    "pa_act_bwd": [_I, _I, _P, _P, _P, _P, _L, _F, _F, _P],
    "pa_softmax_ce_prob_fwd": [_I, _P, _P, _P, _P, _P, _L, _I, _L, _P],
    "pa_softmax_ce_prob_bwd": [_I, _P, _P, _P, _P, _P, _L, _I, _L, _P],
    "pa_cast_any": [_I, _I, _P, _P, _L, _I, _P],
    "pa_strided_gather": [_I, _P, _P, _I, _LP, _LP, _L, _P],
    "pa_random": [_I, _P, _L, _I, _F, _F, ctypes.c_ulonglong, _P],
    "pa_loss_fwd": [_I, _I, _P, _P, _P, _P, _L, _F, _P],
    "pa_loss_bwd": [_I, _I, _P, _P, _P, _P, _P, _L, _L, _F, _P],
    "pa_seq_softmax_fwd": [_I, _P, _P, _P, _L, _P],
    "pa_seq_softmax_bwd": [_I, _P, _P, _P, _P, _L, _P],
    "pa_softmax_ce_fwd": [_I, _P, _P, _P, _P, _P, _L, _I, _L, _P],
    "pa_softmax_ce_bwd": [_I, _P, _P, _P, _P, _P, _P, _L, _I, _L, _F, _P],
    "pa_softmax_fwd": [_I, _P, _P, _L, _I, _I, _P],
    "pa_softmax_bwd": [_I, _P, _P, _P, _L, _I, _I, _P],
    "pa_adamw": [_I, _I, _P, _P, _P, _P, _P, _L, _F, _P, _F, _F, _F, _F, _F, _F, _P, _P, _L, _F, _P, _I, _P],
    "pa_momentum": [_I, _P, _P, _P, _L, _F, _P, _F, _I, _F, _F, _P],
    "pa_bn_running_update": [_I, _P, _P, _P, _P, _I, _L, _F, _F, _P],
    "pa_momentum_p": [_I, _I, _P, _P, _P, _L, _F, _P, _F, _I, _F, _F, _P],
    "pa_sumsq": [_I, _P, _L, _P, _P],
    "pa_sgemm_set_deterministic": [_I],
    "pa_gemm_epi": [_I, _P, _P, _P, _P, _L, _I, _I, _I, _L, _L, _L, _P, _P, _I, _I, _P],
    "pa_sgemm_get_deterministic": [],
    "pa_transpose2d": [_I, _P, _P, _I, _I, _L, _L, _I, _L, _L, _P],
    "pa_flash_attn_fwd": [_P, _P, _P, _P, _P, _LP, _I, _I, _I, _I, _I, _I, _F, _I, _P],
    "pa_fa_bwd_set_variant": [_I],
    "pa_fa_fwd_set_variant": [_I],
    "pa_fa_bwd_get_variant": [],
    "pa_add_attn_fwd": [_P, _P, _P, _P, _P, _P, _L, _P, _I, _I, _I, _I, _P],
    "pa_add_attn_bwd": [_P, _L, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P],
    "pa_lstm_cell_fwd": [_P, _P, _P, _P, _P, _P, _L, _P, _L, _I, _I, _P],
    "pa_lstm_cell_bwd": [_P, _P, _L, _P, _P, _P, _P, _P, _I, _I, _P],
    "pa_lstm_persistent": [_I] + [_P] * 17 + [_I, _I, _I, _P],
    "pa_fa_dq_reduce_rope": [_P, _I, _I, _I, _I, _I, _I, _P, _L, _P, _P, _I, _P],
    "pa_fa_bwd_part_kblk": [_I, _I, _I, _I],
    "pa_conv_gemm": [_P, _P, _P, _P] + [_I] * 17 + [_P],
    "pa_conv_sn": [_P, _P, _P, _P] + [_I] * 17 + [_P, _P, _P],
    "pa_conv_sn_tiles": [_L],
    "pa_conv_sn_acc": [_P, _P, _P, _P] + [_I] * 17 + [_P, _P, _I, _P],
    "pa_conv_gemm_acc": [_P, _P, _P, _P] + [_I] * 18 + [_P],
    "pa_conv_gemm_stats": [_P, _P, _P, _P] + [_I] * 18 + [_P, _P, _P],
    "pa_conv_gemm_bnbwd": [_P, _P, _P, _P] + [_I] * 18 + [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P],
    "pa_conv_sn_bnbwd": [_P, _P, _P] + [_I] * 18 + [_P, _P, _P, _P, _P, _P, _P, _I, _I, _P],
    "pa_momentum_multi": [_P, _I, _L, _F, _P, _F, _I, _F, _P],
    "pa_momentum_multi_entry_bytes": [],
    "pa_momentum_multi_chunk": [],
    "pa_conv_wgrad_sn_ws": [_I] * 9,
    "pa_conv_wgrad_sn": [_P, _P, _P, _P] + [_I] * 16 + [_P],
    "pa_conv_wgrad_sn_ws2": [_I] * 9,
    "pa_conv_wgrad_sn_w": [_P, _P, _P, _I, _P] + [_I] * 16 + [_P],
    "pa_bn_fwd_stats": [_P, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _L, _I, _F, _F, _I, _P, _P],
    "pa_im2col_nhwc": [_P, _P] + [_I] * 15 + [_P],
    "pa_bn_blocks": [_L, _I],
    "pa_bn_fwd_train": [_P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _L, _I, _F, _F, _I, _P, _P],
    "pa_bn_apply": [_P, _P, _P, _P, _P, _P, _I, _L, _I, _I, _P],
    "pa_bn_bwd": [_P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _L, _I, _I, _P, _P],
    "pa_bn_bwd2": [_P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _L, _I, _I, _P, _P],
    "pa_bn_bwd_part": [_P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _L, _I, _I, _P, _P],
    "pa_maxpool_nhwc_fwd": [_P, _P, _P] + [_I] * 12 + [_P],
    "pa_maxpool_nhwc_bwd": [_P, _P, _P] + [_I] * 12 + [_P],
    "pa_gap_nhwc_fwd": [_P, _P, _I, _I, _I, _P],
    "pa_gap_nhwc_bwd": [_P, _P, _I, _I, _I, _P],
    "pa_gemm_set_sched": [_I],
    "pa_gemm_set_persistent": [_I],
    "pa_gemm_set_stagger": [_I],
    "pa_gemm_set_dw1w": [_I],
    "pa_gemm": [_I, _I, _I, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _L, _L, _I, _F, _I, _I, _I, _P, _I, _P],
    "pa_gemm_padded": [_I, _I, _I, _P, _P, _P, _I, _I, _I, _L, _L, _L, _I, _P],
    "pa_splitk_reduce": [_P, _P, _L, _I, _I, _P],
    "pa_moe_gather": [_P, _P, _P, _L, _I, _P],
    "pa_group_tile_table": [_P, _I, _L, _P],
    "pa_clip_coef": [_P, _F, _F, _P, _P],
    "pa_fold_grad": [_I, _P, _P, _L, _I, _P],
    "pa_p2p_alloc": [ctypes.POINTER(_P), ctypes.c_size_t],
    "pa_p2p_free": [_P],
    "pa_p2p_ipc_handle": [_P, _P],
    "pa_p2p_ipc_handle_size": [],
    "pa_p2p_ipc_open": [_P, ctypes.POINTER(_P)],
    "pa_p2p_ipc_close": [_P],
    "pa_p2p_barrier": [_P, _P, _I, _I, ctypes.c_uint, _L, _P, _P],
    "pa_p2p_reduce": [_I, _P, _P, _I, _I, _P, _L, _L, _P, _P],
    "pa_p2p_gather": [_I, _P, _P, _I, _I, _P, _L, _L, _P, _P],
    "pa_p2p_zero": [_P, ctypes.c_size_t],
    "pa_device_count": [ctypes.POINTER(_I)],
    "pa_clear_error": [],
    "pa_one_hot": [_P, _P, _L, _I, _P, _P],
    "pa_pad2d": [_I, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _F, _I, _P],
    "pa_pad2d_bwd": [_I, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "pa_lrn_fwd": [_I, _P, _P, _P, _I, _I, _L, _I, _F, _F, _F, _P],
    "pa_lrn_bwd": [_I, _P, _P, _P, _P, _I, _I, _L, _I, _F, _F, _P],
    "pa_row_conv_fwd": [_I, _P, _P, _P, _P, _L, _I, _I, _P],
    "pa_row_conv_bwd": [_I, _P, _P, _P, _P, _P, _P, _P, _L, _I, _I, _P],
    "pa_argsort_rows": [_I, _P, _P, _P, _L, _I, _I, _P],
    "pa_accuracy": [_P, _P, _L, _I, _P, _P, _P, _P],
    "pa_iou_matrix": [_P, _P, _I, _I, _I, _P, _P],
    "pa_box_coder": [_I, _P, _P, _P, _I, _I, _I, _P, _P],
    "pa_nms_bitmask": [_P, _P, _P, _I, _I, _I, _I, _F, _I, _P, _P],
    "pa_fused_ew_act": [_I, _I, _I, _I, _F, _P, _P, _P, _P, _L, _L, _L, _P],
    "pa_fused_ew_act_bwd": [_I, _I, _I, _I, _F, _P, _P, _P, _P, _P, _L, _L, _L, _P],
    "pa_opt_adamax": [_P, _P, _P, _P, _P, _P, _F, _F, _F, _L, _P],
    "pa_opt_decayed_adagrad": [_P, _P, _P, _P, _F, _F, _L, _P],
    "pa_opt_adadelta": [_P, _P, _P, _P, _F, _F, _L, _P],
    "pa_opt_rmsprop": [_P, _P, _P, _P, _P, _P, _F, _F, _F, _L, _P],
    "pa_opt_ftrl": [_P, _P, _P, _P, _P, _F, _F, _F, _L, _P],
    "pa_opt_proximal": [_P, _P, _P, _P, _F, _F, _L, _P],
    "pa_opt_lars": [_P, _P, _P, _P, _P, _F, _F, _F, _L, _P],
    "pa_ctc_loss": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P],
    "pa_roi_pool_fwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _P, _P, _P],
    "pa_roi_pool_bwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P],
    "pa_edit_distance": [_P, _P, _P, _P, _I, _I, _P, _I, _P, _P],
    "pa_ctc_align": [_P, _P, _I, _I, _I, _P, _P, _P],
    "pa_mean_iou_hist": [_P, _P, _L, _I, _I, _P, _P, _P],
    "pa_fake_quant": [_P, _L, _I, _P, _I, _I, _P, _P, _P, _P],
    "pa_isfinite": [_P, _L, _I, _P, _P],
    "pa_seq_pad": [_P, _P, _I, _I, _L, _P, _I, _I, _P, _P],
    "pa_seq_unpad": [_P, _P, _I, _I, _L, _L, _I, _P, _P],
    "pa_seq_scale": [_P, _P, _I, _L, _L, _P, _I, _P],
    "pa_dwconv_fwd": [_P, _P, _P, _P] + [_I] * 13 + [_P],
    "pa_dwconv_dgrad": [_P, _P, _P] + [_I] * 13 + [_P],
    "pa_dwconv_wgrad": [_P, _P, _P] + [_I] * 13 + [_P],
    "pa_copy2d": [_P, ctypes.c_size_t, _P, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, _P],
    "pa_can_access_peer": [_I, _I, ctypes.POINTER(_I)],
    "pa_enable_peer_access": [_I, _I],
    "pa_memcpy_peer_async": [_P, _I, _P, _I, ctypes.c_size_t, _P],
    "pa_mem_info": [_I, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)],
    "pa_p2p_copy": [_P, _P, ctypes.c_size_t, _P],
    "pa_ce_mean_fwd": [_P, _P, _L, _I, _L, _P, _P, _P],
    "pa_ce_mean_bwd_rows": [_P, _P, _P, _L, _P],
    "pa_binary": [_I, _I, _P, _P, _P, _L, _I, _P, _P, _P, _I, _P],
    "pa_reduce": [_I, _I, _P, _P, _L, _L, _L, _P],
    "pa_dropout": [_I, _P, _P, _P, _L, _F, _F, ctypes.c_ulonglong, ctypes.c_ulonglong, _P],
    "pa_mask_mul": [_I, _P, _P, _P, _L, _F, _P],
    "pa_topk": [_I, _P, _P, _P, _L, _I, _I, _P],
    "pa_sgd": [_I, _P, _P, _P, _L, _P],
    "pa_sgd_sparse": [_P, _P, _P, _P, _L, _I, _P],
    "pa_adagrad": [_P, _P, _P, _P, _L, _F, _P],
    "pa_gather_rows": [_I, _P, _P, _P, _L, _I, _F, _P],
    "pa_scatter_add_rows": [_P, _P, _P, _L, _I, _P],
    "pa_seq_pool": [_I, _P, _P, _P, _P, _I, _I, _I, _F, _P],
    "pa_seq_pool_grad": [_I, _P, _P, _P, _P, _I, _I, _I, _P],
    "pa_gru_gate": [_P, _P, _P, _P, _P, _L, _I, _P],
    "pa_gru_out": [_P, _P, _P, _P, _P, _L, _P],
    "pa_gru_out_bwd": [_P, _P, _P, _P, _P, _P, _P, _L, _P],
    "pa_gru_gate_bwd": [_P, _P, _P, _P, _P, _P, _P, _L, _I, _P],
    "pa_gemm_f8": [_I, _P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _L, _I, _F, _I, _P, _I, _P],
    "pa_quant_rows_f8": [_P, _L, _P, _L, _P, _L, _I, _P],
    "pa_quant_cols_t_f8": [_P, _P, _P, _I, _I, _I, _P],
    "pa_group_cat_offsets": [_I, _P, _I, _P, _P, _P],
    "pa_group_image": [_I, _I, _P, _P, _P, _P, _P, _I, _L, _I, _P, _P, _L, _P, _P],
    "pa_fa_gqa_fold": [_P, _P, _P, _P, _L, _I, _I, _I, _L, _P],
    "pa_gemm_splitk_sum": [_P, _I, _L, _I, _P, _I, _P, _L, _P],
    "pa_moe_reduce": [_P, _P, _P, _P, _L, _I, _I, _P],
    "pa_moe_combine_bwd": [_P, _P, _P, _P, _P, _P, _L, _I, _I, _P],
    "pa_moe_route": [_P, _L, _I, _I, _I, _L, _P, _P, _P, _P, _P, _P],
    "pa_moe_frac": [_P, _L, _I, _I, _P, _P],
    "pa_moe_gate_bwd": [_P, _P, _P, _P, _P, _P, _P, _L, _I, _I, _I, _P, _P],
    "pa_sgemm": [_P, _L, _L, _P, _L, _L, _P, _L, _L, _L, _L, _I, _I, _L, _L, _L, _L, _L, _L, _I, _L, _L, _P, _L, _F,
                 _F, _I, _P, _P],
    "pa_vol2col": [_I, _P, _P, _P, _I, _P],
    "pa_col2vol": [_P, _P, _P, _I, _I, _P],
    "pa_chan_sum": [_P, _P, _I, _I, _L, _I, _P],
    "pa_pool_fwd": [_I, _P, _P, _P, _L, _P, _I, _I, _P],
    "pa_pool_bwd": [_I, _P, _P, _P, _L, _P, _I, _I, _P],
    "pa_unpool": [_I, _I, _P, _P, _P, _L, _L, _L, _P, _P],
    "pa_bn_nchw_groups": [_I, _L],
    "pa_bn_nchw_fwd": [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _L, _F, _F, _I, _I, _I, _P],
    "pa_bn_nchw_bwd": [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _L, _I, _P],
    "pa_prior_box": [_P, _P, _P, _P, _I, _I, _I, _F, _F, _F, _F, _F, _I, _P, _P],
    "pa_anchor_generator": [_P, _P, _P, _P, _I, _I, _I, _F, _F, _F, _P, _P],
    "pa_polygon_box_transform": [_P, _P, _L, _I, _I, _I, _P],
    "pa_target_assign": [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _L, _F, _P],
    "pa_cross_entropy": [_I, _I, _P, _P, _P, _P, _P, _L, _I, _L, _P],
    "pa_cos_sim": [_I, _P, _P, _P, _P, _P, _L, _I, _I, _P],
    "pa_cos_sim_bwd": [_I, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _I, _P],
    "pa_interp": [_I, _I, _P, _P, _L, _I, _I, _I, _I, _I, _I, _P],
    "pa_conv_shift": [_I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P],
    "pa_lstm_unit": [_I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _F, _P],
    "pa_maxout": [_I, _P, _P, _P, _P, _I, _I, _I, _L, _P],
    "pa_flash_attn_bwd": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _LP, _I, _I, _I, _I, _I, _I, _F, _I, _P, _P],
    "pa_fa_bwd_split_ok": [_I, _I, _I, _I, _I, _I, _LP],
    "pa_fa_bwd_split": [_P] * 10 + [_LP, _I, _I, _I, _I, _I, _I, _F, _I, _P, _P, _P],
}


def lib():
    """Load (building on first use if hipcc is available) the kernel library."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = _build.KERNEL_LIB
        if not os.path.exists(path):
            try:
                _build.build_kernels()
            except Exception as e:  # pragma: no cover - exercised only without a prebuilt lib
                raise RuntimeError(
                    f"paddle_amd HIP kernel library missing ({path}) and could not be built: {e}. "
                    "Run `python -m paddle_amd._build` (or __graft_entry__.build()).") from e
        L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _I
        if os.environ.get("FLAGS_cudnn_deterministic", "0").lower() in ("1", "true", "yes", "on"):
            L.pa_sgemm_set_deterministic(1)  # no float-atomic split-K anywhere
        _lib = L
        return _lib


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_GET_DEVICE = getattr(torch._C, "_cuda_getDevice", None)


_FAST = []


def fastops():
    """The C++ launch entry for flat elementwise ops (csrc/fastops, built by
    _build.build_fastops), or None when it is not built / loadable."""
    if not _FAST:
        mod = None
        path = os.path.join(os.path.dirname(_build.KERNEL_LIB), "pa_fastops.so")
        if os.path.exists(path) and os.environ.get("FLAGS_fastops", "1") not in ("0", "false", "False"):
            try:
                import importlib.machinery
                import importlib.util

                lib()  # the kernel library first (RTLD_GLOBAL): the extension links it
                loader = importlib.machinery.ExtensionFileLoader("pa_fastops", path)
                spec = importlib.util.spec_from_file_location("pa_fastops", path, loader=loader)
                mod = importlib.util.module_from_spec(spec)
                loader.exec_module(mod)
            except Exception:  # pragma: no cover - a stale / ABI-mismatched build
                mod = None
        _FAST.append(mod)
    return _FAST[0]


def stream():
    """torch's current HIP stream of the current device, as a raw handle (the C
    accessor: no Stream object per call -- this runs once per kernel launch)."""
    if _RAW_STREAM is not None and _GET_DEVICE is not None:
        return _RAW_STREAM(_GET_DEVICE())
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    """Device pointer of ``t`` for a kernel-library call.  A host tensor here would be
    dereferenced by a HIP kernel (an illegal-address fault that takes the GPU down):
    refuse it on the host instead (pinned host buffers are device-accessible)."""
    if t is None:
        return None
    if not t.is_cuda and t.numel() > 0 and not t.is_pinned():
        raise RuntimeError(f"paddle_amd kernel argument is a host tensor ({tuple(t.shape)}, {t.dtype}); "
                           "every operand of a GPU op must live on the device")
    return _P(t.data_ptr())


def dt(t) -> int:
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    raise TypeError(f"paddle_amd kernels support float32/bfloat16, got {t.dtype}")


class EnforceError(RuntimeError):
    """A failed HIP call or launch (reference platform/enforce.h PADDLE_ENFORCE with
    the cuda/nccl error decoders): carries the HIP error code and its name."""

    def __init__(self, what, rc):
        self.rc = rc
        super().__init__(f"paddle_amd kernel {what} failed: {error_name(rc)} ({rc}): {error_string(rc)}")


def error_name(rc: int) -> str:
    try:
        f = lib().pa_error_name
        f.restype, f.argtypes = ctypes.c_char_p, [_I]
        return (f(int(rc)) or b"?").decode()
    except Exception:  # library unavailable: the code alone
        return f"hipError {rc}"


def error_string(rc: int) -> str:
    try:
        f = lib().pa_error_string
        f.restype, f.argtypes = ctypes.c_char_p, [_I]
        return (f(int(rc)) or b"").decode()
    except Exception:
        return ""


def check(rc: int, what: str):
    if rc != 0:
        try:  # reset the sticky last-error so later (torch) launch checks stay clean
            lib().pa_clear_error()
        except Exception:
            pass
        raise EnforceError(what, rc)


def call(name: str, *args):
    rc = getattr(lib(), name)(*args)
    check(rc, name)
