"""Thin torch-tensor wrappers around the C ABI (include/dctae.h).

Every function enqueues work on torch's current stream of the tensors'
device and returns device tensors; nothing here computes on the CPU.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import FECfg, Images, LFQCfg, Norm, PackedOut, Packing, VQCfg, i32, i64, ptr


@dataclass(frozen=True)
class FEParams:
    channels: int = 3
    patch_size: int = 14
    max_patch_h: int = 32
    max_patch_w: int = 32
    max_seq_len: int = 3072
    channel_importances: Tuple[float, float, float] = (8.0, 1.0, 1.0)
    magnitude_weight: float = 0.1

    def c(self, max_seq_len: Optional[int] = None) -> FECfg:
        ci = tuple(float(x) for x in self.channel_importances)
        if len(ci) != 3:
            raise AssertionError("channel_importances must have 3 entries")
        return FECfg(self.channels, self.patch_size, self.max_patch_h, self.max_patch_w,
                     int(max_seq_len if max_seq_len is not None else self.max_seq_len),
                     (C.c_float * 3)(*ci), float(self.magnitude_weight))


@dataclass
class NormState:
    median: torch.Tensor   # (C, mh, mw, P*P) fp32 on device, contiguous
    b: torch.Tensor
    eps: float = 1e-6
    min_val: float = -6.0
    max_val: float = 6.0
    thr: Optional[torch.Tensor] = None   # LFQ-bit thresholds (norm_thresholds), optional

    def c(self) -> Norm:
        return Norm(C.c_void_p(self.median.data_ptr()), C.c_void_p(self.b.data_ptr()), float(self.eps),
                    float(self.min_val), float(self.max_val), ptr(self.thr))


def norm_thresholds(norm: NormState) -> torch.Tensor:
    """thr = smallest fp32 x with PatchNorm(x) > 0 per table element (exact;
    see dctae_norm_thresholds)."""
    dev = _check_dev(norm.median, norm.b)
    ctx = _lib.context(dev)
    thr = torch.empty_like(norm.median)
    n0 = NormState(norm.median, norm.b, norm.eps, norm.min_val, norm.max_val, None)
    rc = ctx.lib.dctae_norm_thresholds(ctx.h, C.byref(n0.c()), thr.numel(), ptr(thr), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_norm_thresholds")
    return thr


def set_fft(enable: bool, device=None):
    ctx = _lib.context(device)
    ctx.check(ctx.lib.dctae_set_fft(ctx.h, int(bool(enable))), "dctae_set_fft")


def set_option(key: str, value: int, device=None):
    ctx = _lib.context(device)
    ctx.check(ctx.lib.dctae_set_option(ctx.h, key.encode(), int(value)), f"dctae_set_option({key})")


def set_chunk_bytes(nbytes: int, device=None):
    ctx = _lib.context(device)
    ctx.check(ctx.lib.dctae_set_chunk_bytes(ctx.h, int(nbytes)), "dctae_set_chunk_bytes")


def _check_dev(*ts):
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise _lib.DCTAEUnavailable("the MI355X path needs HIP device tensors (got a CPU tensor)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise AssertionError("tensors on different devices")
    return dev


def image_set(images: Sequence[torch.Tensor]) -> Tuple[Images, torch.device, list]:
    """Describe a list of (3,H,W) fp32 contiguous device images by a base
    pointer and element offsets (no copies)."""
    imgs = [im if (im.dtype == torch.float32 and im.is_contiguous()) else im.float().contiguous()
            for im in images]
    dev = _check_dev(*imgs)
    for im in imgs:
        if im.dim() != 3:
            raise AssertionError(f"expected a (c, h, w) image, got {tuple(im.shape)}")
    ptrs = [im.data_ptr() for im in imgs]
    base = min(ptrs) if ptrs else 0
    offs = [(p - base) // 4 for p in ptrs]
    hw = []
    for im in imgs:
        hw += [im.shape[1], im.shape[2]]
    keep = [imgs, i64(offs), i32(hw)]
    desc = Images(C.c_void_p(base), C.cast(keep[1], C.POINTER(C.c_int64)), C.cast(keep[2], C.POINTER(C.c_int32)),
                  len(imgs))
    return desc, dev, keep


def batch_image_set(x: torch.Tensor) -> Tuple[Images, torch.device, list]:
    """(B,3,H,W) fp32 contiguous device tensor."""
    if x.dim() != 4:
        raise AssertionError("expected (B, c, h, w)")
    x = x if (x.dtype == torch.float32 and x.is_contiguous()) else x.float().contiguous()
    dev = _check_dev(x)
    B, c, H, W = x.shape
    per = c * H * W
    keep = [x, i64([i * per for i in range(B)]), i32([H, W] * B)]
    desc = Images(C.c_void_p(x.data_ptr()), C.cast(keep[1], C.POINTER(C.c_int64)),
                  C.cast(keep[2], C.POINTER(C.c_int32)), B)
    return desc, dev, keep


def encode(imgs_desc: Images, dev: torch.device, p: FEParams, plan, n_rows: int, seq_len: int,
           norm: Optional[NormState], lfq: Optional[LFQCfg], want_codes=True, want_patches=False,
           want_raw=False, want_scores=False, out=None):
    """dctae_encode: returns dict of packed device tensors."""
    ctx = _lib.context(dev)
    S = seq_len
    PP = p.patch_size ** 2
    o = out or {}
    def alloc(name, shape, dtype):
        t = o.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype or t.device != dev:
            t = torch.empty(shape, dtype=dtype, device=dev)
            o[name] = t
        return t
    res = {
        "positions": alloc("positions", (n_rows, S, 2), torch.long),
        "channels": alloc("channels", (n_rows, S), torch.long),
        "image_ids": alloc("image_ids", (n_rows, S), torch.long),
        "key_pad_mask": alloc("key_pad_mask", (n_rows, S), torch.bool),
    }
    if want_codes:
        res["codes"] = alloc("codes", (n_rows, S, lfq.num_codebooks), torch.long)
    if want_patches:
        res["patches"] = alloc("patches", (n_rows, S, PP), torch.float32)
    if want_raw:
        res["raw"] = alloc("raw", (n_rows, S, PP), torch.float32)
    if want_scores:
        res["scores"] = alloc("scores", (n_rows, S), torch.float32)
    pk_keep = [i32(plan.row), i32(plan.col), i32(plan.k), i32(plan.local_id), i32(plan.row_len)]
    pk = Packing(*[C.cast(a, C.POINTER(C.c_int32)) for a in pk_keep], n_rows)
    po = PackedOut(ptr(res.get("codes")), ptr(res["positions"]), ptr(res["channels"]), ptr(res["image_ids"]),
                   ptr(res["key_pad_mask"]), ptr(res.get("patches")), ptr(res.get("raw")), ptr(res.get("scores")))
    nc = norm.c() if norm is not None else None
    rc = ctx.lib.dctae_encode(ctx.h, C.byref(p.c(S)), C.byref(imgs_desc), C.byref(pk),
                              C.byref(nc) if nc is not None else None,
                              C.byref(lfq) if lfq is not None else None, C.byref(po), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_encode")
    return res


def norm_apply(x: torch.Tensor, channels: torch.Tensor, positions: torch.Tensor, norm: NormState, p: FEParams,
               inverse: bool) -> torch.Tensor:
    dev = _check_dev(x, channels, positions, norm.median, norm.b)
    ctx = _lib.context(dev)
    PP = p.patch_size ** 2
    if x.shape[-1] != PP:
        raise AssertionError(f"token dim {x.shape[-1]} != patch_size**2")
    xs = x.float().contiguous()
    ch = channels.long().contiguous()
    pos = positions.long().contiguous()
    n = xs.numel() // PP
    if ch.numel() != n or pos.numel() != 2 * n:
        raise AssertionError("channels/positions do not match patches")
    y = torch.empty_like(xs)
    fn = ctx.lib.dctae_norm_inverse if inverse else ctx.lib.dctae_norm_forward
    rc = fn(ctx.h, C.byref(norm.c()), p.patch_size, p.max_patch_h, p.max_patch_w, ptr(xs), ptr(ch), ptr(pos), n,
            ptr(y), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_norm")
    return y


def _stats_inputs(x, channels, positions, key_pad, p: FEParams):
    dev = _check_dev(x, channels, positions)
    PP = p.patch_size ** 2
    if x.shape[-1] != PP:
        raise AssertionError(f"token dim {x.shape[-1]} != patch_size**2")
    xs = x.float().contiguous()
    n = xs.numel() // PP
    ch = channels.long().contiguous()
    pos = positions.long().contiguous()
    if ch.numel() != n or pos.numel() != 2 * n:
        raise AssertionError("channels/positions do not match patches")
    kp = None
    if key_pad is not None:
        kp = key_pad.to(device=dev, dtype=torch.bool).contiguous()
        if kp.numel() != n:
            raise AssertionError("key_pad_mask does not match patches")
    return dev, xs, ch, pos, kp, n


def norm_batch_stats(x, channels, positions, key_pad, p: FEParams):
    """patchnorm.py:104-130 on the GPU: (batch_n (C,mh,mw), batch_median (C,mh,mw,P*P))."""
    dev, xs, ch, pos, kp, n = _stats_inputs(x, channels, positions, key_pad, p)
    ctx = _lib.context(dev)
    PP = p.patch_size ** 2
    bn = torch.empty(p.channels, p.max_patch_h, p.max_patch_w, device=dev)
    bm = torch.empty(p.channels, p.max_patch_h, p.max_patch_w, PP, device=dev)
    rc = ctx.lib.dctae_norm_batch_stats(ctx.h, p.patch_size, p.channels, p.max_patch_h, p.max_patch_w, ptr(xs),
                                        ptr(ch), ptr(pos), ptr(kp), n, ptr(bn), ptr(bm), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_norm_batch_stats")
    return bn, bm


def norm_batch_mad(x, channels, positions, key_pad, median, p: FEParams):
    """patchnorm.py:140-144 on the GPU: batch_b around `median` (C,mh,mw,P*P)."""
    dev, xs, ch, pos, kp, n = _stats_inputs(x, channels, positions, key_pad, p)
    ctx = _lib.context(dev)
    med = median.float().contiguous()
    bb = torch.empty_like(med)
    rc = ctx.lib.dctae_norm_batch_mad(ctx.h, p.patch_size, p.channels, p.max_patch_h, p.max_patch_w, ptr(xs),
                                      ptr(ch), ptr(pos), ptr(kp), n, ptr(med), ptr(bb), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_norm_batch_mad")
    return bb


def norm_merge_(table, batch, n, batch_n, n_update: bool):
    """patchnorm.py:135-138 / 146-150 in place: table <- (table*n + batch*bn)/clamp(n+bn,1); n += bn."""
    dev = _check_dev(table, batch, n, batch_n)
    for t in (table, batch, n, batch_n):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise AssertionError("PatchNorm tables must be contiguous float32")
    cells = n.numel()
    PP = table.numel() // max(1, cells)
    ctx = _lib.context(dev)
    rc = ctx.lib.dctae_norm_merge(ctx.h, cells, PP, ptr(table), ptr(batch), ptr(n), ptr(batch_n), int(n_update),
                                  _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_norm_merge")


def norm_train_step(x, channels, positions, key_pad, n, median, b, p: FEParams, want_output=True):
    """patchnorm.py:101-155 in one call: updates n / median / b in place,
    returns x with the pad rows zeroed (or None)."""
    dev, xs, ch, pos, kp, ntok = _stats_inputs(x, channels, positions, key_pad, p)
    _check_dev(n, median, b)
    ctx = _lib.context(dev)
    y = torch.empty_like(xs) if want_output else None
    st = NormState(median, b)
    rc = ctx.lib.dctae_norm_train_step(ctx.h, C.byref(st.c()), ptr(n), p.patch_size, p.channels, p.max_patch_h,
                                       p.max_patch_w, ptr(xs), ptr(ch), ptr(pos), ptr(kp), ntok, ptr(y),
                                       _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_norm_train_step")
    return y


def check_device_errors(dev):
    ctx = _lib.context(dev)
    ctx.check(ctx.lib.dctae_check_device_errors(ctx.h, _lib.stream_ptr(dev)), "device index check")


def lfq_forward(x: torch.Tensor, cfg: LFQCfg, want_quantized=True):
    dev = _check_dev(x)
    ctx = _lib.context(dev)
    xs = x.float().contiguous()
    d = cfg.codebook_dim * cfg.num_codebooks
    if xs.shape[-1] != d:
        raise AssertionError(f"expected dimension of {d} but received {xs.shape[-1]}")
    n = xs.numel() // d
    q = torch.empty_like(xs) if want_quantized else None
    idx = torch.empty((*xs.shape[:-1], cfg.num_codebooks), dtype=torch.long, device=dev)
    rc = ctx.lib.dctae_lfq_forward(ctx.h, C.byref(cfg), ptr(xs), n, ptr(q), ptr(idx), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_lfq_forward")
    return q, idx


def lfq_codes(idx: torch.Tensor, cfg: LFQCfg) -> torch.Tensor:
    dev = _check_dev(idx)
    ctx = _lib.context(dev)
    ii = idx.long().contiguous()
    if ii.shape[-1] != cfg.num_codebooks:
        raise AssertionError("last dim of indices must be num_codebooks")
    n = ii.numel() // cfg.num_codebooks
    out = torch.empty((*ii.shape[:-1], cfg.num_codebooks * cfg.codebook_dim), dtype=torch.float32, device=dev)
    rc = ctx.lib.dctae_lfq_indices_to_codes(ctx.h, C.byref(cfg), ptr(ii), n, ptr(out), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_lfq_indices_to_codes")
    return out


def lfq_project_in(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], cfg: LFQCfg,
                   x_bound: Optional[float] = None) -> torch.Tensor:
    """LFQ.forward's indices with project_in fused (dctae_lfq_project_in):
    x (..., dim) -> (..., num_codebooks) int64.  w / b: project_in's fp32
    weight (ncb*cd, dim) and bias on x's device.  x_bound: the caller's bound
    |x| <= x_bound (dctae_lfq_project_in_bounded: the fp16 kernels)."""
    return lfq_project_in_into(x, w, b, cfg, None, x_bound)


def lfq_project_in_into(x, w, b, cfg: LFQCfg, idx: Optional[torch.Tensor],
                        x_bound: Optional[float] = None) -> torch.Tensor:
    dev = _check_dev(x, w, b)
    ctx = _lib.context(dev)
    xs = x.float().contiguous()
    dim = xs.shape[-1]
    n = xs.numel() // dim
    shape = (*xs.shape[:-1], cfg.num_codebooks)
    if idx is None or idx.shape != shape or idx.dtype != torch.long or not idx.is_contiguous() or idx.device != dev:
        idx = torch.empty(shape, dtype=torch.long, device=dev)
    if x_bound is not None:
        rc = ctx.lib.dctae_lfq_project_in_bounded(ctx.h, C.byref(cfg), ptr(xs), n, dim, ptr(w), ptr(b),
                                                  float(x_bound), ptr(idx), _lib.stream_ptr(dev))
        ctx.check(rc, "dctae_lfq_project_in_bounded")
        return idx
    rc = ctx.lib.dctae_lfq_project_in(ctx.h, C.byref(cfg), ptr(xs), n, dim, ptr(w), ptr(b), ptr(idx),
                                      _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_lfq_project_in")
    return idx


def lfq_project_out(idx: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], cfg: LFQCfg) -> torch.Tensor:
    """LFQ.indices_to_codes with project_out fused (dctae_lfq_project_out):
    idx (..., num_codebooks) -> (..., dim) fp32; w (dim, ncb*cd), b (dim)."""
    dev = _check_dev(idx, w, b)
    ctx = _lib.context(dev)
    ii = idx.long().contiguous()
    if ii.shape[-1] != cfg.num_codebooks:
        raise AssertionError("last dim of indices must be num_codebooks")
    dim = w.shape[0]
    n = ii.numel() // cfg.num_codebooks
    out = torch.empty((*ii.shape[:-1], dim), dtype=torch.float32, device=dev)
    rc = ctx.lib.dctae_lfq_project_out(ctx.h, C.byref(cfg), ptr(ii), n, dim, ptr(w), ptr(b), ptr(out),
                                       _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_lfq_project_out")
    return out


def lfq_project_out_inverse_norm(idx: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], cfg: LFQCfg,
                                 norm: NormState, p: FEParams, channels: torch.Tensor,
                                 positions: torch.Tensor) -> torch.Tensor:
    """LFQ.indices_to_codes (project_out) + PatchNorm.inverse_norm in one kernel
    (dctae_lfq_project_out_inverse_norm): idx (..., ncb) -> (..., P*P) fp32."""
    dev = _check_dev(idx, w, b, channels, positions, norm.median, norm.b)
    ctx = _lib.context(dev)
    ii = idx.long().contiguous()
    if ii.shape[-1] != cfg.num_codebooks:
        raise AssertionError("last dim of indices must be num_codebooks")
    dim = w.shape[0]
    if dim != p.patch_size ** 2:
        raise AssertionError(f"project_out dim {dim} != patch_size**2")
    n = ii.numel() // cfg.num_codebooks
    ch = channels.long().contiguous()
    pos = positions.long().contiguous()
    if ch.numel() != n or pos.numel() != 2 * n:
        raise AssertionError("channels/positions do not match the indices")
    tshape = (3, p.max_patch_h, p.max_patch_w, dim)
    for t in (norm.median, norm.b):
        if tuple(t.shape) != tshape or not t.is_contiguous() or t.dtype != torch.float32:
            raise AssertionError(f"PatchNorm tables must be contiguous fp32 {tshape}, got {tuple(t.shape)}")
    out = torch.empty((*ii.shape[:-1], dim), dtype=torch.float32, device=dev)
    rc = ctx.lib.dctae_lfq_project_out_inverse_norm(ctx.h, C.byref(cfg), ptr(ii), n, dim, ptr(w), ptr(b),
                                                    C.byref(norm.c()), p.max_patch_h, p.max_patch_w, ptr(ch),
                                                    ptr(pos), ptr(out), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_lfq_project_out_inverse_norm")
    return out


def vq_forward(cfg: VQCfg, x: torch.Tensor, mask: Optional[torch.Tensor], want_quantized=True):
    """x (n, dim) fp32 contiguous on the device; mask (n) bool or None.
    Returns quantize (n, dim) (None unless wanted) and indices (n, heads)."""
    dev = _check_dev(x)
    ctx = _lib.context(dev)
    if x.dtype != torch.float32 or not x.is_contiguous() or x.ndim != 2 or x.shape[1] != cfg.dim:
        raise AssertionError(f"VectorQuantize input must be contiguous fp32 (n, {cfg.dim})")
    n = x.shape[0]
    m = None
    if mask is not None:
        if mask.shape != (n,):
            raise AssertionError("mask must be (n,)")
        m = mask.to(device=dev, dtype=torch.uint8).contiguous()
    q = torch.empty_like(x) if want_quantized else None
    idx = torch.empty((n, cfg.heads), dtype=torch.long, device=dev)
    rc = ctx.lib.dctae_vq_forward(ctx.h, C.byref(cfg), ptr(x), ptr(m), n, ptr(q), ptr(idx), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_vq_forward")
    return q, idx


def vq_from_indices(cfg: VQCfg, idx: torch.Tensor, project_out: bool) -> torch.Tensor:
    """idx (n, heads) -> codes (n, heads*codebook_dim) or project_out(codes) (n, dim)."""
    dev = _check_dev(idx)
    ctx = _lib.context(dev)
    ii = idx.long().contiguous()
    if ii.ndim != 2 or ii.shape[1] != cfg.heads:
        raise AssertionError("indices must be (n, heads)")
    n = ii.shape[0]
    width = cfg.dim if project_out else cfg.heads * cfg.codebook_dim
    out = torch.empty((n, width), dtype=torch.float32, device=dev)
    fn = ctx.lib.dctae_vq_output_from_indices if project_out else ctx.lib.dctae_vq_codes_from_indices
    rc = fn(ctx.h, C.byref(cfg), ptr(ii), n, ptr(out), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_vq_from_indices")
    check_device_errors(dev)
    return out


def decode(p: FEParams, ids: torch.Tensor, key_pad: torch.Tensor, positions: torch.Tensor, channels: torch.Tensor,
           patch_sizes: Sequence, original_sizes: Sequence, codes: Optional[torch.Tensor] = None,
           patches: Optional[torch.Tensor] = None, norm: Optional[NormState] = None,
           lfq: Optional[LFQCfg] = None, normed: bool = False) -> List[torch.Tensor]:
    """dctae_decode; returns a list of (3, H, W) fp32 device images.  normed:
    patches are PatchNorm outputs and the inverse_norm runs inside the decode
    (dctae_decode_normed; norm required, no codes)."""
    dev = _check_dev(ids, key_pad, positions, channels, codes, patches)
    ctx = _lib.context(dev)
    R, S = ids.shape
    ids_c = ids.long().contiguous()
    kp = key_pad.to(torch.bool).contiguous()
    pos = positions.long().contiguous()
    ch = channels.long().contiguous()
    # image enumeration: rows in order, ids ascending (FE:619-633); host view
    ids_h = ids_c.cpu()
    lut_w = int(ids_h.max().item()) + 1 if ids_h.numel() else 1
    lut = [-1] * (R * lut_w)
    n_img = 0
    for r in range(R):
        for im in torch.unique(ids_h[r]).tolist():
            lut[r * lut_w + im] = n_img
            n_img += 1
    if n_img > len(patch_sizes) or n_img > len(original_sizes):
        raise IndexError("more images in the batch than patch_sizes / original_sizes entries")
    hw, phw, offs = [], [], []
    total = 0
    for i in range(n_img):
        h, w = (int(v) for v in original_sizes[i])
        ph, pw = (int(v) for v in patch_sizes[i])
        hw += [h, w]
        phw += [ph, pw]
        offs.append(total)
        total += p.channels * h * w
    out = torch.empty(total, dtype=torch.float32, device=dev)
    keep = [i32(lut), i32(hw), i64(offs), i32(phw)]
    cc = codes.long().contiguous() if codes is not None else None
    pp = patches.float().contiguous() if patches is not None else None
    nc = norm.c() if norm is not None else None
    if normed:
        if nc is None or codes is not None:
            raise AssertionError("normed decode needs the PatchNorm state and patches (no codes)")
        rc = ctx.lib.dctae_decode_normed(ctx.h, C.byref(p.c(S)), R, C.cast(keep[0], C.POINTER(C.c_int32)), lut_w,
                                         n_img, C.cast(keep[1], C.POINTER(C.c_int32)),
                                         C.cast(keep[2], C.POINTER(C.c_int64)), C.cast(keep[3], C.POINTER(C.c_int32)),
                                         ptr(ids_c), ptr(kp), ptr(pos), ptr(ch), C.byref(nc), ptr(pp), ptr(out),
                                         _lib.stream_ptr(dev))
        ctx.check(rc, "dctae_decode_normed")
        check_device_errors(dev)
    else:
        rc = ctx.lib.dctae_decode(ctx.h, C.byref(p.c(S)), R, C.cast(keep[0], C.POINTER(C.c_int32)), lut_w, n_img,
                                  C.cast(keep[1], C.POINTER(C.c_int32)), C.cast(keep[2], C.POINTER(C.c_int64)),
                                  C.cast(keep[3], C.POINTER(C.c_int32)), ptr(ids_c), ptr(kp), ptr(pos), ptr(ch),
                                  C.byref(nc) if nc is not None else None, C.byref(lfq) if lfq is not None else None,
                                  ptr(cc), ptr(pp), ptr(out), _lib.stream_ptr(dev))
        ctx.check(rc, "dctae_decode")
    imgs = []
    for i in range(n_img):
        h, w = hw[2 * i], hw[2 * i + 1]
        imgs.append(out[offs[i]: offs[i] + p.channels * h * w].view(p.channels, h, w))
    return imgs


def dct2(x: torch.Tensor, inverse: bool, color: bool) -> torch.Tensor:
    """dctae_dct2 on a (3, H, W) or (B, 3, H, W) fp32 device tensor: full-image
    orthonormal DCT-II of rgb_to_ipt(x) (FE._transform_image_in, FE:129-142) or
    ipt_to_rgb of the DCT-III (FE._transform_image_out, FE:144-152); color=False
    is util.dct2 / util.idct2 alone (util.py:333-338)."""
    one = x.dim() == 3
    xb = x[None] if one else x
    if xb.dim() != 4 or xb.shape[1] != 3:
        raise AssertionError(f"expected (3, h, w) or (b, 3, h, w), got {tuple(x.shape)}")
    xb = xb if (xb.dtype == torch.float32 and xb.is_contiguous()) else xb.float().contiguous()
    dev = _check_dev(xb)
    ctx = _lib.context(dev)
    y = torch.empty_like(xb)
    B, _, H, W = xb.shape
    color = int(color) if not isinstance(color, bool) else int(color)   # 0 / 1, or 2 / 3: fp16 / bf16 colour
    rc = ctx.lib.dctae_dct2(ctx.h, ptr(xb), B, H, W, int(bool(inverse)), color, ptr(y),
                            _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_dct2")
    return y[0] if one else y


def patch_spectrum(x: torch.Tensor, p: FEParams, k: int):
    """dctae_patch_spectrum: FE._patch_image (FE:364-452) of a cropped (3, h, w)
    spectrum on the device -> (patches (k, P*P), positions (k, 2), channels (k))."""
    x = x if (x.dtype == torch.float32 and x.is_contiguous()) else x.float().contiguous()
    dev = _check_dev(x)
    if x.dim() != 3:
        raise AssertionError(f"expected a (c, h, w) spectrum, got {tuple(x.shape)}")
    ctx = _lib.context(dev)
    P = p.patch_size
    patches = torch.empty((k, P * P), dtype=torch.float32, device=dev)
    pos = torch.empty((k, 2), dtype=torch.long, device=dev)
    ch = torch.empty((k,), dtype=torch.long, device=dev)
    cfg = p.c(p.max_seq_len)
    rc = ctx.lib.dctae_patch_spectrum(ctx.h, C.byref(cfg), ptr(x), x.shape[1], x.shape[2], int(k), ptr(patches),
                                      ptr(pos), ptr(ch), None, _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_patch_spectrum")
    return patches, pos, ch


def synth_images(n: int, h: int, w: int, seed: int, first_index: int = 0, device=None) -> torch.Tensor:
    """(n, 3, h, w) counter-RNG images generated on the device (oracle/rng.py hash)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    ctx = _lib.context(dev)
    out = torch.empty((n, 3, h, w), dtype=torch.float32, device=dev)
    rc = ctx.lib.dctae_synth_images(ctx.h, C.c_uint64(seed), first_index, n, h, w, ptr(out), _lib.stream_ptr(dev))
    ctx.check(rc, "dctae_synth_images")
    return out
