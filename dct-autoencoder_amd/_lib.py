"""ctypes binding of libdctae.so (the C ABI in include/dctae.h).

The product path has no fallback: if the library or a HIP device is missing,
every op raises ``DCTAEUnavailable``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Dict, Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# DCTAE_LIBRARY: another build of the same ABI (e.g. a profiling variant)
LIB_PATH = os.environ.get("DCTAE_LIBRARY") or os.path.join(_HERE, "libdctae.so")
ABI_VERSION = 1


class DCTAEUnavailable(RuntimeError):
    pass


class DCTAEError(RuntimeError):
    pass


# ---- struct mirrors of include/dctae.h ------------------------------------


class FECfg(C.Structure):
    _fields_ = [("channels", C.c_int32), ("patch_size", C.c_int32), ("max_patch_h", C.c_int32),
                ("max_patch_w", C.c_int32), ("max_seq_len", C.c_int32),
                ("channel_importances", C.c_float * 3), ("magnitude_weight", C.c_float)]


class Norm(C.Structure):
    _fields_ = [("median_dev", C.c_void_p), ("b_dev", C.c_void_p), ("eps", C.c_float),
                ("min_val", C.c_float), ("max_val", C.c_float), ("thr_dev", C.c_void_p)]


class LFQCfg(C.Structure):
    _fields_ = [("codebook_dim", C.c_int32), ("num_codebooks", C.c_int32), ("codebook_scale", C.c_float)]


class Images(C.Structure):
    _fields_ = [("rgb_dev", C.c_void_p), ("img_off", C.POINTER(C.c_int64)), ("hw", C.POINTER(C.c_int32)),
                ("n_img", C.c_int32)]


class Packing(C.Structure):
    _fields_ = [("row", C.POINTER(C.c_int32)), ("col", C.POINTER(C.c_int32)), ("k", C.POINTER(C.c_int32)),
                ("local_id", C.POINTER(C.c_int32)), ("row_len", C.POINTER(C.c_int32)), ("n_rows", C.c_int32)]


class PackedOut(C.Structure):
    _fields_ = [("codes_dev", C.c_void_p), ("positions_dev", C.c_void_p), ("channels_dev", C.c_void_p),
                ("image_ids_dev", C.c_void_p), ("key_pad_dev", C.c_void_p), ("patches_dev", C.c_void_p),
                ("raw_patches_dev", C.c_void_p), ("scores_dev", C.c_void_p)]


class VQCfg(C.Structure):
    _fields_ = [("dim", C.c_int32), ("heads", C.c_int32), ("codebook_dim", C.c_int32),
                ("codebook_size", C.c_int32), ("affine", C.c_int32), ("affine_decay", C.c_float),
                ("w_in_dev", C.c_void_p), ("b_in_dev", C.c_void_p), ("w_out_dev", C.c_void_p),
                ("b_out_dev", C.c_void_p), ("embed_dev", C.c_void_p), ("codebook_mean_dev", C.c_void_p),
                ("codebook_variance_dev", C.c_void_p), ("batch_mean_dev", C.c_void_p),
                ("batch_variance_dev", C.c_void_p), ("batch_initted_dev", C.c_void_p)]


_P = C.c_void_p
_SIGS = {
    "dctae_abi_version": ([], C.c_int),
    "dctae_ctx_create": ([C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "dctae_ctx_destroy": ([_P], C.c_int),
    "dctae_last_error": ([_P], C.c_char_p),
    "dctae_set_color_matrices": ([_P, _P, _P, _P, _P], C.c_int),
    "dctae_encode": ([_P, C.POINTER(FECfg), C.POINTER(Images), C.POINTER(Packing), C.POINTER(Norm),
                      C.POINTER(LFQCfg), C.POINTER(PackedOut), _P], C.c_int),
    "dctae_encode_lfq_proj": ([_P, C.POINTER(FECfg), C.POINTER(Images), C.POINTER(Packing), C.POINTER(Norm),
                               C.POINTER(LFQCfg), _P, _P, C.POINTER(PackedOut), _P], C.c_int),
    "dctae_spectrum_tokens": ([_P, C.POINTER(FECfg), C.POINTER(Images), C.POINTER(C.c_int64), _P, _P, _P],
                              C.c_int),
    "dctae_dct2": ([_P, _P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P], C.c_int),
    "dctae_patch_spectrum": ([_P, C.POINTER(FECfg), _P, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P, _P],
                             C.c_int),
    "dctae_norm_forward": ([_P, C.POINTER(Norm), C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, C.c_int64, _P, _P],
                           C.c_int),
    "dctae_norm_inverse": ([_P, C.POINTER(Norm), C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, C.c_int64, _P, _P],
                           C.c_int),
    "dctae_lfq_forward": ([_P, C.POINTER(LFQCfg), _P, C.c_int64, _P, _P, _P], C.c_int),
    "dctae_lfq_indices_to_codes": ([_P, C.POINTER(LFQCfg), _P, C.c_int64, _P, _P], C.c_int),
    "dctae_lfq_project_in": ([_P, C.POINTER(LFQCfg), _P, C.c_int64, C.c_int32, _P, _P, _P, _P], C.c_int),
    "dctae_lfq_project_in_bounded": ([_P, C.POINTER(LFQCfg), _P, C.c_int64, C.c_int32, _P, _P, C.c_float, _P, _P],
                                     C.c_int),
    "dctae_lfq_project_out": ([_P, C.POINTER(LFQCfg), _P, C.c_int64, C.c_int32, _P, _P, _P, _P], C.c_int),
    "dctae_lfq_project_out_inverse_norm": ([_P, C.POINTER(LFQCfg), _P, C.c_int64, C.c_int32, _P, _P, C.POINTER(Norm),
                                            C.c_int32, C.c_int32, _P, _P, _P, _P], C.c_int),
    "dctae_decode": ([_P, C.POINTER(FECfg), C.c_int32, C.POINTER(C.c_int32), C.c_int32, C.c_int32,
                      C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int32), _P, _P, _P, _P,
                      C.POINTER(Norm), C.POINTER(LFQCfg), _P, _P, _P, _P], C.c_int),
    "dctae_decode_normed": ([_P, C.POINTER(FECfg), C.c_int32, C.POINTER(C.c_int32), C.c_int32, C.c_int32,
                             C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int32), _P, _P, _P, _P,
                             C.POINTER(Norm), _P, _P, _P], C.c_int),
    "dctae_vq_forward": ([_P, C.POINTER(VQCfg), _P, _P, C.c_int64, _P, _P, _P], C.c_int),
    "dctae_vq_codes_from_indices": ([_P, C.POINTER(VQCfg), _P, C.c_int64, _P, _P], C.c_int),
    "dctae_vq_output_from_indices": ([_P, C.POINTER(VQCfg), _P, C.c_int64, _P, _P], C.c_int),
    "dctae_check_device_errors": ([_P, _P], C.c_int),
    "dctae_synth_images": ([_P, C.c_uint64, C.c_int64, C.c_int32, C.c_int32, C.c_int32, _P, _P], C.c_int),
    "dctae_set_timing": ([_P, C.c_int], C.c_int),
    "dctae_timing_collect": ([_P], C.c_int),
    "dctae_timing_get": ([_P, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.POINTER(C.c_int64)],
                         C.c_int),
    "dctae_timing_reset": ([_P], C.c_int),
    "dctae_set_workspace_limit": ([_P, C.c_int64], C.c_int),
    "dctae_norm_thresholds": ([_P, C.POINTER(Norm), C.c_int64, _P, _P], C.c_int),
    "dctae_set_fft": ([_P, C.c_int], C.c_int),
    "dctae_set_chunk_bytes": ([_P, C.c_int64], C.c_int),
    "dctae_set_option": ([_P, C.c_char_p, C.c_int64], C.c_int),
    "dctae_norm_batch_stats": ([_P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P, C.c_int64, _P, _P,
                                _P], C.c_int),
    "dctae_norm_batch_mad": ([_P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P, C.c_int64, _P, _P,
                              _P], C.c_int),
    "dctae_norm_merge": ([_P, C.c_int32, C.c_int32, _P, _P, _P, _P, C.c_int32, _P], C.c_int),
    "dctae_norm_train_step": ([_P, C.POINTER(Norm), _P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P,
                               C.c_int64, _P, _P], C.c_int),
    # DCTAutoencoder transformer operators
    "dctae_model_linear": ([_P, C.c_int64, C.c_int32, C.c_int32, _P, C.c_int64, _P, C.c_int32, C.c_int64, _P,
                            C.c_int32, _P, C.c_int64, _P], C.c_int),
    "dctae_model_attention": ([_P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P, C.c_int64, _P],
                              C.c_int),
    "dctae_model_layernorm": ([_P, C.c_int64, C.c_int32, _P, C.c_int64, _P, _P, C.c_float, _P, C.c_int64, _P],
                              C.c_int),
    "dctae_model_embed_norm": ([_P, C.c_int64, C.c_int32, _P, C.c_int64, _P, _P, C.c_float, _P, _P, _P, _P, _P, _P,
                                C.c_int64, _P], C.c_int),
    "dctae_model_pos_add": ([_P, C.c_int64, C.c_int32, _P, C.c_int64, _P, _P, _P, _P, _P, _P], C.c_int),
    "dctae_model_to_bf16": ([_P, C.c_int64, C.c_int32, _P, C.c_int64, C.c_int32, _P, _P], C.c_int),
    "dctae_model_lfq": ([_P, C.c_int64, C.c_int32, C.c_int32, C.c_float, _P, C.c_int64, _P, _P, _P, C.c_int64, _P],
                        C.c_int),
}

_lib = None
_lib_lock = threading.Lock()


def load_library():
    """dlopen libdctae.so and bind every symbol of include/dctae.h (no GPU needed)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise DCTAEUnavailable(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C csrc)")
        lib = C.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        v = lib.dctae_abi_version()
        if v != ABI_VERSION:
            raise DCTAEUnavailable(f"libdctae ABI {v} != {ABI_VERSION}")
        _lib = lib
        return lib


class Context:
    """One dctae_ctx per (device, thread)."""

    def __init__(self, device: int):
        lib = load_library()
        h = C.c_void_p()
        rc = lib.dctae_ctx_create(int(device), C.byref(h))
        if rc != 0:
            raise DCTAEUnavailable(f"dctae_ctx_create(device={device}) failed ({rc}): "
                                   f"{lib.dctae_last_error(None).decode()}")
        self.lib = lib
        self.h = h
        self.device = device
        from . import color
        m = color.matrices()
        keep = [m[k].contiguous().float().cpu() for k in ("rgb2lms", "lms2ipt", "ipt2lms", "lms2rgb")]
        self.check(lib.dctae_set_color_matrices(h, *[C.c_void_p(t.data_ptr()) for t in keep]))

    def check(self, rc: int, what: str = ""):
        if rc != 0:
            msg = self.lib.dctae_last_error(self.h).decode()
            if rc == -1:
                raise AssertionError(f"{what}: {msg}")
            raise DCTAEError(f"{what} failed ({rc}): {msg}")

    def __del__(self):
        try:
            if getattr(self, "h", None) is not None and self.h.value:
                self.lib.dctae_ctx_destroy(self.h)
        except Exception:
            pass


_ctx_by_key: Dict = {}


def context(device: Optional[torch.device] = None) -> Context:
    if not torch.cuda.is_available():
        raise DCTAEUnavailable("no HIP device visible (torch.cuda.is_available() is False)")
    if device is None:
        idx = torch.cuda.current_device()
    else:
        device = torch.device(device)
        if device.type != "cuda":
            raise DCTAEUnavailable(f"tensor on {device}: the MI355X path needs HIP device tensors")
        idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, threading.get_ident())
    ctx = _ctx_by_key.get(key)
    if ctx is None:
        ctx = Context(idx)
        _ctx_by_key[key] = ctx
    return ctx


def stream_ptr(device=None) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t: Optional[torch.Tensor]) -> C.c_void_p:
    return C.c_void_p(t.data_ptr() if t is not None else 0)


def i32(vals):
    arr = (C.c_int32 * max(1, len(vals)))(*[int(v) for v in vals])
    return arr


def i64(vals):
    arr = (C.c_int64 * max(1, len(vals)))(*[int(v) for v in vals])
    return arr
