"""ctypes binding of librf.so (include/rf_api.h).

The product path has NO fallback: if the library is missing or no GPU is visible, every operator
raises. Build the library with ``python -c "import __graft_entry__ as g; g.build()"`` (or
``make -C recommendflow_amd/csrc``).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RF_LIB") or os.path.normpath(os.path.join(_HERE, "..", "lib", "librf.so"))  # RF_LIB: diagnostics only

RF_OK, RF_EINVAL, RF_EHIP, RF_EOOB = 0, -1, -2, -3
DT_F32, DT_BF16, DT_F16 = 0, 1, 2
COMB = {"sum": 0, "avg": 1, "max": 2, "min": 3, "first": 4, "last": 5, "null": 6, "cls": 4}
FLAG_MASK_PADDING, FLAG_EMIT_IDX, FLAG_SINGLE_TOKEN, FLAG_TREE_REDUCE, FLAG_SPEC_ROWS = 0x1, 0x2, 0x4, 0x10, 0x20
ACT = {None: 0, "none": 0, "linear": 0, "gelu": 1, "relu": 2, "selu": 3, "softmax": 4}

_lock = threading.Lock()
_lib = None

_i32, _i64, _u64, _vp, _f32 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_float
_SIGS = {
    "rf_abi_version": (_i32, []),
    "rf_last_error": (ctypes.c_char_p, []),
    "rf_siphash_bucket": (ctypes.c_int, [_vp, _vp, _i64, _u64, _u64, _i64, _i32, _vp, _vp]),
    "rf_fused_hash_embed_fwd": (ctypes.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _i32, _vp, _i32, _i64, _i32, _vp, _i32, _i64, _i32, _vp, _vp]),
    "rf_embedding_bag_fwd": (ctypes.c_int, [_vp, _i32, _i32, _i64, _vp, _i32, _i64, _i32, _i32, _vp, _i32, _i64, _i64, _vp]),
    "rf_table_init_uniform": (ctypes.c_int, [_vp, _i32, _i64, _i32, _i64, _i64, _u64, _f32, _f32, _vp]),
    "rf_esim_soft_attention_fwd": (ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, _i32, _i64, _i64, _vp, _i64, _i64, _vp, _vp]),
    "rf_esim_soft_attention_idx_fwd": (ctypes.c_int, [_vp, _i32, _vp, _vp, _i64, _i64, _i32, _i32, _i32, _i32, _i64, _i64, _vp, _i64,
                                                      _i64, _vp]),
    "rf_esim_gather_fwd": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32, _vp, _i64, _i64, _vp]),
    "rf_single_token_ids_fwd": (ctypes.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _i32, _i64, _vp, _i32, _vp]),
    "rf_single_token_ids_multi_fwd": (ctypes.c_int, [_vp, _i32, _vp]),
    "rf_norm_fwd": (ctypes.c_int, [_vp, _i64, _i32, _i64, _i32, _f32, _vp, _vp, _vp, _vp, _vp, _i32, _i64, _vp]),
    "rf_linear_fwd": (ctypes.c_int, [_vp, _i32, _i64, _i32, _i64, _vp, _i32, _vp, _i32, _vp, _i64, _vp]),
    "rf_dense_head_fwd": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _i32, _vp, _i32, _vp, _i64, _vp]),
    "rf_linear_stats_fwd": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _vp, _i32, _vp, _i64, _vp, _vp]),
    "rf_linear_lnfold_fwd": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _vp, _vp, _vp, _f32, _i32, _vp, _i64,
                                            _vp]),
    "rf_mlp2_small_fwd": (ctypes.c_int, [_vp, _i64, _i32, _i64, _f32, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _i32,
                                         _i32, _vp, _i64, _vp]),
    "rf_mlp2_small_stats_fwd": (ctypes.c_int, [_vp, _i64, _i32, _i64, _f32, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp,
                                               _i32, _i32, _vp, _i64, _vp, _i32, _i32, _vp]),
    "rf_linear_lnfold_stats_fwd": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _vp, _vp, _vp, _f32, _i32, _vp, _i64,
                                                  _vp, _vp]),
    "rf_linear_lnfold_head_ws_bytes": (ctypes.c_size_t, [_i64, _i32]),
    "rf_linear_lnfold_head_fwd": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _i32, _vp, _vp, _vp, _f32, _i32, _vp, _i64,
                                                 _vp, _i32, _vp, _i32, _vp, _i64, _vp, ctypes.c_size_t, _vp]),
    "rf_esim_gather_stats_fwd": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32, _vp, _i64, _i64,
                                                _vp, _i32, _i32, _vp]),
    "rf_sdpa_fwd": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp]),
    "rf_bucketize_ws_bytes": (ctypes.c_size_t, [_i64, _i32]),
    "rf_bucketize_owner": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_gather_rows": (ctypes.c_int, [_vp, _i64, _vp, _i32, _i64, _i32, _vp, _vp]),
    "rf_hash_rows": (ctypes.c_int, [_vp, _i32, _vp, _vp, _vp, _i32, _vp, _vp]),
    "rf_route_ws_bytes": (ctypes.c_size_t, [_i64, _i32, _i64]),
    "rf_route_rows": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_pool_rows_fwd": (ctypes.c_int, [_vp, _i32, _vp, _vp, _i32, _i64, _vp, _vp, _vp, _i32, _i32, _vp, _i32, _i64, _i32, _vp]),
    "rf_pp_ws_bytes": (ctypes.c_size_t, [_i64]),
    "rf_pp_plan": (ctypes.c_int, [_vp, _i32, _vp, _vp, _i32, _i64, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp,
                                  ctypes.c_size_t, _vp]),
    "rf_pp_heads": (ctypes.c_int, [_vp, _i64, _vp, _i32, _vp, _vp, _i64, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_pp_owner_pool": (ctypes.c_int, [_vp, _i32, _vp, _i64, _vp, _i64, _vp, _i32, _i64, _i32, _vp, _vp]),
    "rf_pp_combine": (ctypes.c_int, [_vp, _i32, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _i32, _vp, _i32, _i64, _vp]),
    "rf_route_hash_ws_bytes": (ctypes.c_size_t, [_i64, _i32, _i64]),
    "rf_route_hash_build": (ctypes.c_int, [_vp, _i64, _i32, _i32, _i64, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_route_hash_finish": (ctypes.c_int, [_i64, _i32, _i64, _i64, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_route_hash_build_tokens": (ctypes.c_int, [_vp, _i32, _vp, _vp, _vp, _i32, _i64, _vp, _i32, _i32, _i32, _i64, _vp,
                                                  _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_embed_bwd_ws_bytes": (ctypes.c_size_t, [_i64, _i32, _i64]),
    "rf_fused_hash_embed_bwd": (ctypes.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _i32, _i64, _vp, _i64, _i32, _vp, _vp, _i64,
                                               _i32, _vp, _vp, _vp, _i64, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_pool_rows_bwd": (ctypes.c_int, [_vp, _i32, _vp, _vp, _i32, _i64, _i64, _vp, _vp, _i64, _i32, _vp, _vp, _i64, _i32,
                                        _vp, _vp, _vp, _i64, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_segment_sum_ws_bytes": (ctypes.c_size_t, [_i64, _i64]),
    "rf_segment_sum_rows": (ctypes.c_int, [_vp, _vp, _i64, _i32, _i64, _vp, _vp, _i64, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_adam_ws_bytes": (ctypes.c_size_t, [_i64, _i32]),
    "rf_adam_apply": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _i64, _f32, _f32, _f32, _f32, _i32, _vp,
                                     ctypes.c_size_t, _vp]),
    "rf_cosine_rows_fwd": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i32, _i32, _f32, _vp, _vp, _vp]),
    "rf_cosine_rows_bwd": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i32, _i32, _f32, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                                          _i64, _vp]),
    "rf_loss_ws_bytes": (ctypes.c_size_t, [_i32]),
    "rf_cosent_loss": (ctypes.c_int, [_vp, _vp, _i32, _f32, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_softmax_ce_loss": (ctypes.c_int, [_vp, _i64, _vp, _i32, _i32, _vp, _vp, _i64, _vp, _i64, _vp, ctypes.c_size_t, _vp]),
    "rf_esim_train_ws_bytes": (ctypes.c_size_t, [_i32, _i32, _i32]),
    "rf_esim_train_fwd_f32": (ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, _i64, _i64, _vp, _i64, _i64, _vp, _vp]),
    "rf_esim_train_bwd_f32": (ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp,
                                             _vp, _vp, _i64, _i64, _vp, ctypes.c_size_t, _vp]),
    "rf_act_dropout_fwd": (ctypes.c_int, [_vp, _i64, _i64, _i32, _i32, _f32, ctypes.c_uint64, _vp, _i64, _vp]),
    "rf_act_dropout_bwd": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i32, _i32, _f32, ctypes.c_uint64, _vp, _i64, _vp, _vp,
                                          ctypes.c_size_t, _vp]),
    "rf_layernorm_bwd_ws_bytes": (ctypes.c_size_t, [_i64, _i32]),
    "rf_layernorm_bwd": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i32, _vp, _f32, _vp, _i64, _vp, _vp, _vp, ctypes.c_size_t,
                                        _vp]),
    "rf_inbatch_ce_loss": (ctypes.c_int, [_vp, _i64, _vp, _i32, _f32, _vp, _vp, _i64, _vp, ctypes.c_size_t, _vp]),
    "rf_vocab_capacity": (_i64, [_i64]),
    "rf_vocab_build": (ctypes.c_int, [_i32, _vp, _vp, _i64, _vp, _i64]),
    "rf_lookup_ids": (ctypes.c_int, [_i32, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp]),
    "rf_bucketize_ids": (ctypes.c_int, [_vp, _vp, _i32, _i32, _i32, _i32, _vp, _i32, _f32, _vp, _vp]),
    "rf_attention_fusion_fwd": (ctypes.c_int, [_vp, _i32, _i32, _i32, _i64, _vp, _i32, _vp, _i64, _vp, _vp]),
    "rf_linear_splitk_ws_bytes": (ctypes.c_size_t, [_i32, _i64, _i32, _i32]),
    "rf_linear_splitk_fwd": (ctypes.c_int, [_vp, _i32, _i64, _i32, _i64, _vp, _i32, _vp, _i32, _vp, _i64, _vp,
                                            ctypes.c_size_t, _vp]),
    "rf_fused_hash_embed_bwd_plan": (ctypes.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _i32, _i64, _i64, _i32, _i64, _i32,
                                                    _vp, _i64, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_fused_hash_embed_bwd_reduce": (ctypes.c_int, [_vp, _i32, _vp, _vp, _vp, _vp, _i32, _i64, _vp, _i64, _i32, _vp,
                                                      _vp, _i64, _i32, _vp, _vp, _vp, _i64, _vp, _vp, ctypes.c_size_t,
                                                      _vp]),
    "rf_adam_dense": (_i32, [_vp, _vp, _vp, _vp, _i64, _f32, _f32, _f32, _f32, _vp]),
    "rf_adam_dense_multi": (_i32, [_vp, _i32, _i64, _f32, _f32, _f32, _f32, _vp]),
    "rf_adam_apply_current": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _i64, _f32, _f32, _f32, _f32, _vp,
                                             _i32, _vp]),
    "rf_adam_replay": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _i64, _vp, _i32, _i32, _vp, _f32, _f32, _f32,
                                      _vp]),
    "rf_adam_untouched": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _i64, _f32, _f32, _f32, _f32, _vp,
                                         ctypes.c_size_t, _vp]),
    "rf_gemm_f32_ws_bytes": (ctypes.c_size_t, [_i64, _i64, _i64]),
    "rf_gemm_f32_grouped_ws_bytes": (ctypes.c_size_t, [_vp, _i32]),
    "rf_gemm_f32_grouped": (ctypes.c_int, [_vp, _i32, _i32, _i32, _vp, ctypes.c_size_t, _vp]),
    "rf_gemm_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i64, _i32, _i64, _i64, _i64, _vp, _i32, _vp, _i64, _vp,
                                   ctypes.c_size_t, _vp]),
    "rf_tower_ws_bytes": (ctypes.c_size_t, [_i64, _i32]),
    "rf_col_stats": (ctypes.c_int, [_vp, _i64, _i32, _i64, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "rf_bn_fold": (ctypes.c_int, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp]),
    "rf_dropout_fwd": (ctypes.c_int, [_vp, _i64, _i32, _i64, _f32, ctypes.c_uint64, _vp, _i64, _vp]),
    "rf_selu_dropout_bwd": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i32, _f32, ctypes.c_uint64, _vp, _i64, _vp, _vp,
                                           ctypes.c_size_t, _vp]),
    "rf_bn_fold_grad": (ctypes.c_int, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _vp]),
    "rf_bn_bwd": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i32, _vp, _vp, _vp, _f32, _vp, _i64, _vp, _vp, _vp,
                                 ctypes.c_size_t, _vp]),
    "rf_stream_copy": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp]),
    "rf_gather_probe": (ctypes.c_int, [_vp, _i64, _i32, _i64, _i32, ctypes.c_uint64, _vp, _vp, _vp]),
    "rf_topk_merge": (ctypes.c_int, [_vp, _i64, _i32, _i32, _i32, _i64, _vp, _vp, _i32, _i64, _vp, _vp, _i64, _vp]),
    "rf_topk_merge_idx": (ctypes.c_int, [_vp, _vp, _i64, _i32, _i32, _i32, _vp, _vp, _i32, _i64, _vp, _vp, _i64, _vp]),
    "rf_ip_candidates_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i32, _i32, _vp, _i32, _vp, _vp, _vp, _i64, _vp]),
    "rf_ip_rescore_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _i32, _vp, _vp, _i32, _vp]),
    "rf_ip_candidates_bf16": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i64, _vp]),
}
EXPORTED = tuple(_SIGS)
# include/rf_diag.h: tools-only entry points (not the production ABI)
_DIAG_SIGS = {"rf_diag_fused_hash_embed_fwd": _SIGS["rf_fused_hash_embed_fwd"],
              "rf_diag_esim_gather_stamped": (ctypes.c_int, _SIGS["rf_esim_gather_fwd"][1][:-1] + [_vp, _i32, _vp])}
DIAG_EXPORTED = tuple(_DIAG_SIGS)
DIAG_ABLATIONS = 0x7000  # bits 12-14: accepted only by rf_diag_fused_hash_embed_fwd


class IdsTask(ctypes.Structure):
    """include/rf_api.h rf_ids_task (rf_single_token_ids_multi_fwd)."""
    _fields_ = [("slots", _vp), ("tok_bytes", _vp), ("tok_off", _vp), ("bag_off", _vp), ("lmax", _vp), ("ids", _vp),
                ("table_rows", _i64), ("n_slots", _i32), ("batch", _i32), ("flags", _i32), ("reserved", _i32)]


class GemmProblem(ctypes.Structure):
    """include/rf_api.h rf_gemm_f32_problem."""
    _fields_ = [("A", _vp), ("lda", _i64), ("B", _vp), ("ldb", _i64), ("C", _vp), ("ldc", _i64), ("bias", _vp),
                ("M", _i64), ("N", _i64), ("K", _i64), ("act", _i32), ("reserved", _i32)]


class RFError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load librf.so (no GPU needed to load). Raises RFError if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RFError(f"librf.so not found at {path}: build it first (make -C recommendflow_amd/csrc)")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in list(_SIGS.items()) + list(_DIAG_SIGS.items()):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.rf_abi_version() != 1:
            raise RFError(f"librf.so ABI version {lib.rf_abi_version()} != 1")
        _lib = lib
        return lib


def require_gpu():
    import torch

    if not torch.cuda.is_available():
        raise RFError("recommendflow_amd operators need a ROCm GPU (torch.cuda.is_available() is False); "
                      "there is no CPU fallback")


def check(rc: int, what: str):
    if rc != RF_OK:
        msg = load().rf_last_error().decode(errors="replace")
        kind = {RF_EINVAL: "invalid argument", RF_EHIP: "HIP error", RF_EOOB: "out of range"}.get(rc, str(rc))
        if rc == RF_EINVAL:
            raise ValueError(f"{what}: {kind}: {msg}")
        raise RFError(f"{what}: {kind}: {msg}")


def stream_ptr(stream=None) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None for None)."""
    return None if t is None else int(t.data_ptr())


def call(name: str, *args):
    fn = getattr(load(), name)
    rc = fn(*args)
    check(rc, name)
    return rc


def torch_dtype_code(dtype) -> int:
    import torch

    if dtype == torch.float32:
        return DT_F32
    if dtype == torch.bfloat16:
        return DT_BF16
    if dtype == torch.float16:
        return DT_F16
    raise ValueError(f"unsupported dtype {dtype}")
