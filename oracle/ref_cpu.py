"""CPU restatement of the reference hot path — TEST INFRASTRUCTURE ONLY.

This module is the *checker* for the MI355X implementation.  It restates, in
float32 PyTorch-CPU code written for this repo, the algorithm of the reference
``theAdamColton/dct-autoencoder`` on the feature-extraction hot path
(SURVEY.md §8(a) rows a1-a13).  Every function cites the reference file:line it
follows (paths relative to the reference repo root).

Rules (see DESIGN.md "Oracle"):
  * only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import this module;
  * the product package (``dct-autoencoder_amd/``) never imports it;
  * it is pinned against golden vectors produced by running the reference
    itself in the build container (``tests/golden/gen_golden.py``) and, for
    the DCT, against ``scipy.fft.dctn(type=2, norm='ortho')`` in float64.

Third-party boundary: the reference's DCT comes from ``torch_dct==0.1.6``
(reference requirements.txt:13, called from dct_autoencoder/util.py:333-338).
That package is not vendored in the reference; ``dct_1d``/``idct_1d`` below
restate its published algorithm (Makhoul's FFT-based DCT-II / DCT-III with
'ortho' scaling).

Documented deviation: the reference orders tokens with an *unstable*
``sort(descending=True)`` (feature_extraction_dct_autoencoder.py:418); its tie
order is an implementation detail of the CPU sort.  The oracle (and the GPU
path) use the deterministic order (score desc, flat index asc).  Comparisons
against the reference are therefore made per image as a map (c, h, w) -> token.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

# ---------------------------------------------------------------------------
# configuration (reference feature_extraction_dct_autoencoder.py:108-127)
# ---------------------------------------------------------------------------


@dataclass
class FEConfig:
    channels: int = 3
    patch_size: int = 14
    sample_patches_beta: float = 0.0
    max_patch_h: int = 32
    max_patch_w: int = 32
    max_seq_len: int = 3072
    channel_importances: Tuple[float, ...] = (8.0, 1.0, 1.0)
    patch_sample_magnitude_weight: float = 0.1


# ---------------------------------------------------------------------------
# a1 / a12: colour transform (reference util.py:18-97)
# ---------------------------------------------------------------------------

# Published colour-science constants, reference util.py:21-39.
_SRGB_TO_XYZ = ((0.4124564, 0.3575761, 0.1804375),
                (0.2126729, 0.7151522, 0.0721750),
                (0.0193339, 0.1191920, 0.9503041))
_XYZ_TO_LMS = ((0.4002, 0.7076, -0.0807),
               (-0.2280, 1.1500, 0.0612),
               (0.0, 0.0, 0.9184))
_LMS_TO_IPT = ((0.4, 0.4, 0.2),
               (4.455, -4.851, 0.3960),
               (0.8056, 0.3572, -1.1628))
IPT_GAMMA = 0.43  # util.py:43


def color_matrices() -> Dict[str, torch.Tensor]:
    """fp32 matrices exactly as the reference builds them (util.py:40-41, 91)."""
    srgb = torch.tensor(_SRGB_TO_XYZ, dtype=torch.float32)
    hpe = torch.tensor(_XYZ_TO_LMS, dtype=torch.float32)
    ipt = torch.tensor(_LMS_TO_IPT, dtype=torch.float32)
    rgb2lms = hpe @ srgb                      # util.py:40  Trgb2lms = MHPE @ MsRGB
    return {
        "rgb2lms": rgb2lms,
        "lms2rgb": rgb2lms.inverse(),         # util.py:41
        "lms2ipt": ipt,                       # util.py:37
        "ipt2lms": ipt.inverse(),             # util.py:91 (Mipt.inverse())
    }


def _channel_mult(m: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    # util.py:46-47  einsum "i j, ... j h w -> ... i h w"
    return torch.einsum("ij,...jhw->...ihw", m.to(x.dtype), x)


def _signed_pow(x: torch.Tensor, p: float) -> torch.Tensor:
    # util.py:76-78 / 94-96: sign(x) * |x| ** p
    neg = x < 0.0
    y = x.abs() ** p
    y[neg] = -y[neg]
    return y


def rgb_to_ipt(x: torch.Tensor) -> torch.Tensor:
    """reference util.py:70-82"""
    m = color_matrices()
    return _channel_mult(m["lms2ipt"], _signed_pow(_channel_mult(m["rgb2lms"], x), IPT_GAMMA))


def ipt_to_rgb(x: torch.Tensor) -> torch.Tensor:
    """reference util.py:85-97"""
    m = color_matrices()
    return _channel_mult(m["lms2rgb"], _signed_pow(_channel_mult(m["ipt2lms"], x), 1 / IPT_GAMMA))


# ---------------------------------------------------------------------------
# a2 / a12: orthonormal DCT-II / DCT-III, restating torch_dct 0.1.6
# (called from reference util.py:333-338)
# ---------------------------------------------------------------------------


def dct_1d(x: torch.Tensor) -> torch.Tensor:
    """Orthonormal DCT-II over the last dim (torch_dct.dct(x, 'ortho'))."""
    shape = x.shape
    n = shape[-1]
    x = x.contiguous().view(-1, n)
    # Makhoul reordering: even samples ascending, odd samples descending
    v = torch.cat([x[:, ::2], x[:, 1::2].flip([1])], dim=1)
    spec = torch.view_as_real(torch.fft.fft(v, dim=1))
    ang = -torch.arange(n, dtype=x.dtype)[None, :] * np.pi / (2 * n)
    out = spec[:, :, 0] * torch.cos(ang) - spec[:, :, 1] * torch.sin(ang)
    out[:, 0] /= np.sqrt(n) * 2
    out[:, 1:] /= np.sqrt(n / 2) * 2
    return (2 * out).view(*shape)


def idct_1d(y: torch.Tensor) -> torch.Tensor:
    """Orthonormal DCT-III over the last dim (torch_dct.idct(X, 'ortho'))."""
    shape = y.shape
    n = shape[-1]
    yv = y.contiguous().view(-1, n) / 2
    yv[:, 0] *= np.sqrt(n) * 2
    yv[:, 1:] *= np.sqrt(n / 2) * 2
    ang = torch.arange(n, dtype=y.dtype)[None, :] * np.pi / (2 * n)
    wr, wi = torch.cos(ang), torch.sin(ang)
    tr = yv
    ti = torch.cat([yv[:, :1] * 0, -yv.flip([1])[:, :-1]], dim=1)
    vr = tr * wr - ti * wi
    vi = tr * wi + ti * wr
    spec = torch.stack([vr, vi], dim=2)
    v = torch.fft.irfft(torch.view_as_complex(spec), n=n, dim=1)
    out = v.new_zeros(v.shape)
    out[:, ::2] += v[:, : n - (n // 2)]
    out[:, 1::2] += v.flip([1])[:, : n // 2]
    return out.view(*shape)


def dct2(x: torch.Tensor) -> torch.Tensor:
    """reference util.py:333-334 -> torch_dct.dct_2d(x, 'ortho')"""
    return dct_1d(dct_1d(x).transpose(-1, -2)).transpose(-1, -2)


def idct2(x: torch.Tensor) -> torch.Tensor:
    """reference util.py:337-338 -> torch_dct.idct_2d(x, 'ortho')"""
    return idct_1d(idct_1d(x).transpose(-1, -2)).transpose(-1, -2)


def dct_matrix_f64(n: int) -> np.ndarray:
    """C_N[k, m] = s_k cos(pi (2m+1) k / 2N), the exact orthonormal DCT-II matrix."""
    k = np.arange(n)[:, None].astype(np.float64)
    m = np.arange(n)[None, :].astype(np.float64)
    c = np.cos(np.pi * (2 * m + 1) * k / (2 * n)) * np.sqrt(2.0 / n)
    c[0] *= np.sqrt(0.5)
    return c


# ---------------------------------------------------------------------------
# a3 / a4: crop + spectral patching + importance order
# (reference feature_extraction_dct_autoencoder.py:129-177, 312-452)
# ---------------------------------------------------------------------------


def crop_dims(h: int, w: int, patch_size: int) -> Tuple[int, int]:
    """FE:312-345"""
    assert h >= patch_size and w >= patch_size
    ph = max(int(h / patch_size), 1)
    pw = max(int(w / patch_size), 1)
    return ph * patch_size, pw * patch_size


def exp_trunc_dist(beta: float, rng=random) -> float:
    """reference util.py:167-172 (draws from python ``random``)"""
    return -1 / beta * math.log(rng.random())


def num_tokens(h: int, w: int, cfg: FEConfig) -> int:
    ch, cw = crop_dims(h, w, cfg.patch_size)
    ph, pw = ch // cfg.patch_size, cw // cfg.patch_size
    return cfg.channels * min(ph, cfg.max_patch_h) * min(pw, cfg.max_patch_w)


def choose_k(total: int, cfg: FEConfig, rng=random) -> int:
    """FE:429-435"""
    k = total
    if cfg.sample_patches_beta > 0.0:
        k = min(round(exp_trunc_dist(cfg.sample_patches_beta, rng)), k)
        k = max(1, k)
    return min(k, cfg.max_seq_len)


def patch_scores(x: torch.Tensor, cfg: FEConfig):
    """Tokens of a cropped spectrum and their importance scores (FE:364-416).

    x: (c, 14ph, 14pw) fp32.  Returns tokens (T, 196) in flat order
    f = (h*qw + w)*c + ch, positions (T, 2), channels (T,), scores (T,)."""
    c, hh, ww = x.shape
    p = cfg.patch_size
    assert hh % p == 0 and ww % p == 0
    ph, pw = hh // p, ww // p
    # "c (h p1) (w p2) -> (h w) c (p1 p2)"   FE:374-380
    t = x.reshape(c, ph, p, pw, p).permute(1, 3, 0, 2, 4).reshape(ph * pw, c, p * p)
    hi, wi = torch.meshgrid(torch.arange(ph), torch.arange(pw), indexing="ij")
    keep = ((hi < cfg.max_patch_h) & (wi < cfg.max_patch_w)).flatten()   # FE:393
    t = t[keep]
    hi = hi.flatten()[keep]
    wi = wi.flatten()[keep]
    dist = (-1 * (hi + wi)).unsqueeze(-1).expand(-1, c)                   # FE:403-406
    mags = t.abs().amax(-1) * cfg.patch_sample_magnitude_weight          # FE:409-410
    ci = torch.tensor(cfg.channel_importances, dtype=torch.float32)
    scores = (mags + dist / ci).flatten()                                # FE:416-418
    tokens = t.reshape(-1, p * p)
    pos = torch.stack([hi.unsqueeze(-1).expand(-1, c).flatten(),
                       wi.unsqueeze(-1).expand(-1, c).flatten()], -1)
    chans = torch.arange(c).unsqueeze(0).expand(hi.shape[0], -1).flatten()
    return tokens, pos, chans, scores


def patch_image(x: torch.Tensor, cfg: FEConfig, rng=random, stable: bool = True):
    """FE:364-452.  stable=True gives the deterministic (score desc, index asc) order."""
    tokens, pos, chans, scores = patch_scores(x, cfg)
    _, order = scores.sort(dim=0, descending=True, stable=stable)
    k = choose_k(len(order), cfg, rng)
    sel = order[:k]
    return tokens[sel], pos[sel], chans[sel]


def transform_image_in(im: torch.Tensor) -> torch.Tensor:
    """FE:129-142: rgb -> ipt in the input's dtype (FE:135), then .float(),
    dct2 (fp32, CPU) and back to the input's dtype (FE:139-141)."""
    return dct2(rgb_to_ipt(im).float()).to(im.dtype)


def transform_image_out(x: torch.Tensor) -> torch.Tensor:
    """FE:144-152: idct2 -> ipt -> rgb (fp32, CPU)."""
    return ipt_to_rgb(idct2(x.float()))


def preprocess(im: torch.Tensor, cfg: FEConfig, rng=random, stable: bool = True) -> Dict[str, Any]:
    """FE:154-177"""
    y = transform_image_in(im)
    _, h, w = y.shape
    ch, cw = crop_dims(h, w, cfg.patch_size)
    assert y.shape[0] == cfg.channels
    y = y[:, :ch, :cw]                                                      # FE:347-362
    patches, pos, chans = patch_image(y, cfg, rng, stable)
    return dict(patches=patches, positions=pos, channels=chans,
                original_sizes=(h, w),
                patch_sizes=(ch // cfg.patch_size, cw // cfg.patch_size))


# ---------------------------------------------------------------------------
# a5 / a6: greedy packing and collation (FE:179-287, 454-605; util.py:149-164)
# ---------------------------------------------------------------------------


@dataclass
class Batch:
    """Field-for-field the reference DCTPatches (dct_patches.py:6-51)."""
    patches: torch.Tensor
    key_pad_mask: torch.Tensor
    attn_mask: Optional[torch.Tensor]
    batched_image_ids: torch.Tensor
    patch_channels: torch.Tensor
    patch_positions: torch.Tensor
    patch_sizes: List[Tuple[int, int]]
    original_sizes: List[Tuple[int, int]]
    _data: Optional[Dict[str, List[Any]]] = None

    @property
    def h_indices(self):
        return self.patch_positions[..., 0]

    @property
    def w_indices(self):
        return self.patch_positions[..., 1]


@dataclass
class _Groups:
    rows: List[List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]] = field(default_factory=list)
    cur: List[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = field(default_factory=list)
    seq_len: int = 0


def _group(items, cfg: FEConfig, st: _Groups) -> _Groups:
    """FE:454-513 greedy first-fit in arrival order."""
    for patches, pos, chans in items:
        k = patches.shape[0]
        assert k <= cfg.max_patch_h * cfg.max_patch_w * cfg.channels and k <= cfg.max_seq_len
        if st.seq_len + k > cfg.max_seq_len:
            st.rows.append(st.cur)
            st.cur = []
            st.seq_len = 0
        st.cur.append((patches, pos, chans))
        st.seq_len += k
    return st


def _pad_stack(seqs: List[torch.Tensor], s: int) -> torch.Tensor:
    """util.py:149-164"""
    out = torch.zeros((len(seqs), s, *seqs[0].shape[1:]), dtype=seqs[0].dtype)
    for i, q in enumerate(seqs):
        out[i, : q.shape[0]] = q
    return out


def batch_groups(rows, cfg: FEConfig, build_attn_mask: bool = True, **kw) -> Batch:
    """FE:515-605"""
    s = cfg.max_seq_len
    seqs, poss, chs, ids = [], [], [], []
    for row in rows:
        seqs.append(torch.cat([r[0] for r in row], 0))
        poss.append(torch.cat([r[1] for r in row], 0))
        chs.append(torch.cat([r[2] for r in row], 0))
        ids.append(torch.cat([torch.full((r[0].shape[0],), i, dtype=torch.long)
                              for i, r in enumerate(row)]))
    lengths = torch.tensor([q.shape[0] for q in seqs], dtype=torch.long)
    key_pad = lengths[:, None] <= torch.arange(s)[None, :]                # FE:568-576
    bids = _pad_stack(ids, s)
    attn = None
    if build_attn_mask:                                                   # FE:580-584
        attn = (bids[:, None, :, None] == bids[:, None, None, :]) & key_pad[:, None, None, :]
    return Batch(patches=_pad_stack(seqs, s), key_pad_mask=key_pad, attn_mask=attn,
                 batched_image_ids=bids, patch_positions=_pad_stack(poss, s),
                 patch_channels=_pad_stack(chs, s), **kw)


def iter_batches(dataloader, cfg: FEConfig, batch_size: Optional[int] = None,
                 build_attn_mask: bool = True):
    """FE:179-287, including its quirks (trailing partial batch dropped;
    with batch_size=None already-emitted rows are carried into the next batch)."""
    st = None
    sizes_o: List = []
    sizes_p: List = []
    extra: Dict[str, List] = {}
    fixed = {"patches", "positions", "channels", "original_sizes", "patch_sizes"}
    for item in dataloader:
        sizes_o = sizes_o + list(item["original_sizes"])
        sizes_p = sizes_p + list(item["patch_sizes"])
        for k, v in item.items():
            if k not in fixed:
                extra.setdefault(k, []).extend(v)
        st = _group(zip(item["patches"], item["positions"], item["channels"]), cfg, st or _Groups())
        if batch_size is None and st.cur:
            st.rows.append(st.cur)
            st.cur, st.seq_len = [], 0
        if batch_size is None or len(st.rows) > batch_size:
            emit = st.rows[:batch_size]
            st = _Groups(rows=st.rows[batch_size:], cur=st.cur, seq_len=st.seq_len)
            n = sum(len(r) for r in emit)
            o_now, sizes_o = sizes_o[:n], sizes_o[n:]
            p_now, sizes_p = sizes_p[:n], sizes_p[n:]
            x_now = {k: v[:n] for k, v in extra.items()}
            extra = {k: v[n:] for k, v in extra.items()}
            yield batch_groups(emit, cfg, build_attn_mask, original_sizes=o_now,
                               patch_sizes=p_now, _data=x_now)


# ---------------------------------------------------------------------------
# a7 / a10 / a13: PatchNorm (reference patchnorm.py:32-177)
# ---------------------------------------------------------------------------


@dataclass
class NormTables:
    n: torch.Tensor        # (C, H, W)
    median: torch.Tensor   # (C, H, W, P*P)
    b: torch.Tensor        # (C, H, W, P*P)
    eps: float = 1e-6
    max_val: float = 6.0
    min_val: float = -6.0

    @staticmethod
    def fresh(c=3, h=32, w=32, p=14):
        """patchnorm.py:52-69 initial state"""
        return NormTables(torch.zeros(c, h, w), torch.zeros(c, h, w, p * p), torch.ones(c, h, w, p * p))


def norm_forward_eval(t: NormTables, patches, channels, h_idx, w_idx) -> torch.Tensor:
    """patchnorm.py:157-165 (eval / frozen).  Pad tokens are normalised too."""
    med = t.median[channels, h_idx, w_idx]
    std = t.b[channels, h_idx, w_idx] * 2 ** 0.5 + t.eps
    out = (patches - med) / std
    out.clamp_(t.min_val, t.max_val)
    return out


def norm_inverse(t: NormTables, patches, channels, h_idx, w_idx) -> torch.Tensor:
    """patchnorm.py:167-177 (mul then add: no fused multiply-add)."""
    med = t.median[channels, h_idx, w_idx]
    std = t.b[channels, h_idx, w_idx] * 2 ** 0.5 + t.eps
    return patches * std + med


def _scatter_cells(acc: torch.Tensor, ch, hi, wi, vals: Optional[torch.Tensor] = None):
    """patchnorm.py:9-29 scatter_add over (c, h, w) cells, in place."""
    c, h, w, z = acc.shape
    flat = (ch * h * w + hi * w + wi).flatten()
    idx = flat[:, None].expand(-1, z)
    if vals is None:
        vals = torch.ones(idx.shape, dtype=acc.dtype)
    acc.view(c * h * w, z).scatter_add_(0, idx, vals)


def norm_batch_stats(shape, patches, channels, h_idx, w_idx, key_pad_mask):
    """patchnorm.py:104-130: (batch_n, batch_median) of the non-pad tokens;
    batch_median is torch.median(0) (lower median) per occupied cell."""
    keep = ~key_pad_mask
    ch, hi, wi, x = channels[keep], h_idx[keep], w_idx[keep], patches[keep]
    c, h, w, z = shape
    batch_n = torch.zeros(c, h, w, dtype=x.dtype)
    _scatter_cells(batch_n.unsqueeze(-1), ch, hi, wi)
    batch_median = torch.zeros(c, h, w, z, dtype=x.dtype)
    cell = ch * h * w + hi * w + wi
    order = torch.sort(cell, stable=True).indices
    cs = cell[order]
    uniq, counts = torch.unique_consecutive(cs, return_counts=True)
    start = 0
    for u, cnt in zip(uniq.tolist(), counts.tolist()):
        rows = x[order[start:start + cnt]]
        start += cnt
        cc, rem = divmod(u, h * w)
        hh, ww = divmod(rem, w)
        batch_median[cc, hh, ww] = rows.median(0).values                   # lower median
    return batch_n, batch_median


def norm_batch_mad(median, patches, channels, h_idx, w_idx, key_pad_mask, batch_n):
    """patchnorm.py:140-144: scatter_add of |x - median| / clamp(batch_n, 1)."""
    keep = ~key_pad_mask
    ch, hi, wi, x = channels[keep], h_idx[keep], w_idx[keep], patches[keep]
    dist = (x - median[ch, hi, wi]).abs()
    batch_b = torch.zeros_like(median)
    _scatter_cells(batch_b, ch, hi, wi, dist)
    return batch_b / batch_n.unsqueeze(-1).clamp(1)


def norm_merge(table, n, batch, batch_n):
    """patchnorm.py:135-138 / 146-148: (t*n + s*bn) / clamp(n + bn, 1)."""
    return (table * n.unsqueeze(-1) + batch * batch_n.unsqueeze(-1)) / (n + batch_n).clamp(1).unsqueeze(-1)


def norm_train_step(t: NormTables, patches, channels, h_idx, w_idx, key_pad_mask) -> NormTables:
    """patchnorm.py:101-155: one training-mode update of n / median / b."""
    batch_n, batch_median = norm_batch_stats(tuple(t.median.shape), patches, channels, h_idx, w_idx, key_pad_mask)
    median = norm_merge(t.median, t.n, batch_median, batch_n)
    batch_b = norm_batch_mad(median, patches, channels, h_idx, w_idx, key_pad_mask, batch_n)
    b = norm_merge(t.b, t.n, batch_b, batch_n)
    return NormTables(t.n + batch_n, median, b, t.eps, t.max_val, t.min_val)


# ---------------------------------------------------------------------------
# a8 / a9: LFQ eval path (reference lfq.py:35-227)
# ---------------------------------------------------------------------------


@dataclass
class LFQConfig:
    dim: int = 196
    codebook_size: int = 2 ** 14
    num_codebooks: int = 14
    codebook_scale: float = 1.0

    @property
    def codebook_dim(self) -> int:
        return int(math.log2(self.codebook_size))

    @property
    def has_projections(self) -> bool:
        return self.dim != self.codebook_dim * self.num_codebooks

    def bit_weights(self) -> torch.Tensor:
        return 2 ** torch.arange(self.codebook_dim - 1, -1, -1)          # lfq.py:87


def lfq_forward(x: torch.Tensor, cfg: LFQConfig, project_in=None, project_out=None):
    """lfq.py:136-227 eval: returns (quantized, indices int64)."""
    if project_in is not None:
        x = project_in(x)
    b, n, _ = x.shape
    x = x.reshape(b, n, cfg.num_codebooks, cfg.codebook_dim)            # lfq.py:168
    q = torch.where(x > 0, torch.full_like(x, cfg.codebook_scale), torch.full_like(x, -cfg.codebook_scale))
    idx = ((q > 0).int() * cfg.bit_weights().int()).sum(-1)             # lfq.py:187
    q = q.reshape(b, n, -1)
    if project_out is not None:
        q = project_out(q)
    return q, idx


def lfq_indices_to_codes(idx: torch.Tensor, cfg: LFQConfig, project_out=None) -> torch.Tensor:
    """lfq.py:105-134"""
    bits = ((idx[..., None].int() & cfg.bit_weights()) != 0).float()
    codes = bits * cfg.codebook_scale * 2 - cfg.codebook_scale
    codes = codes.reshape(*codes.shape[:-2], -1)
    if project_out is not None:
        codes = project_out(codes)
    return codes


# ---------------------------------------------------------------------------
# VectorQuantize inference (vector_quantize.py), as the model
# builds it (modeling_dct_autoencoder.py:76-77): euclidean codebook shared by
# all heads (separate_codebook_per_head=False), codebook_dim 16, affine_param,
# learnable codebook, kmeans already run (initted), eval mode.
# ---------------------------------------------------------------------------


@dataclass
class VQState:
    w_in: torch.Tensor            # project_in.weight (H*d, dim)          vector_quantize.py:727
    b_in: torch.Tensor            # project_in.bias   (H*d,)
    w_out: torch.Tensor           # project_out.weight (dim, H*d)         vector_quantize.py:728
    b_out: torch.Tensor
    embed: torch.Tensor           # _codebook.embed (1, C, d)             vector_quantize.py:283-288
    codebook_mean: torch.Tensor   # (1, 1, d)                             vector_quantize.py:300-303
    codebook_variance: torch.Tensor
    batch_mean: Optional[torch.Tensor] = None       # (1, 1, d), None until the first forward (:298)
    batch_variance: Optional[torch.Tensor] = None
    heads: int = 1
    decay: float = 0.99           # affine_param_batch_decay (:245)


def vq_update_with_decay(old: Optional[torch.Tensor], new: torch.Tensor, decay: float) -> torch.Tensor:
    """vector_quantize.py:330-343 (no *_needs_init attribute for batch stats)."""
    if old is None:
        return new.detach()
    return old * decay + new.detach() * (1 - decay)


def vq_forward_eval(st: VQState, x: torch.Tensor, mask: Optional[torch.Tensor]):
    """VectorQuantize.forward in eval mode (vector_quantize.py:855-1050) with
    EuclideanCodebook.forward (:424-508).  Returns (quantize (b,n,dim),
    embed_ind (b,n,h) int64, new VQState) — the batch affine statistics are
    updated even in eval mode (:353-359)."""
    b, n, dim = x.shape
    h = st.heads
    d = st.embed.shape[-1]
    xp = torch.nn.functional.linear(x, st.w_in, st.b_in)                 # :883 project_in
    xp = xp.reshape(b, n, h, d).permute(0, 2, 1, 3).reshape(1, b * h, n, d)   # :888 '1 (b h) n d'
    flatten = xp.reshape(1, b * h * n, d)                                 # :444 pack 'h * d'
    data = flatten
    if mask is not None:
        m = mask[:, None, :].expand(b, h, n).reshape(1, b * h * n)          # :447 repeat
        data = flatten[m].reshape(1, -1, d)                               # :367-369
    new_mean = data.mean(dim=1, keepdim=True)                             # :373 reduce mean
    new_var = torch.var(data, dim=1, unbiased=False, keepdim=True)        # :374 var_fn
    bm = vq_update_with_decay(st.batch_mean, new_mean, st.decay)
    bv = vq_update_with_decay(st.batch_variance, new_var, st.decay)
    codebook_std = st.codebook_variance.clamp(min=1e-5).sqrt()           # :458
    batch_std = bv.clamp(min=1e-5).sqrt()                                  # :459
    embed = (st.embed - st.codebook_mean) * (batch_std / codebook_std) + bm   # :460
    x2 = (flatten ** 2).sum(-1)                                           # :29-33 cdist
    y2 = (embed ** 2).sum(-1)
    xy = torch.einsum("b i d, b j d -> b i j", flatten, embed) * -2
    dist = -(x2[..., :, None] + y2[..., None, :] + xy).sqrt()             # :462
    ind = dist.argmax(dim=-1)                                             # :70-90 gumbel_sample, eval
    quant = embed[0][ind[0]]                                              # :219-223 batched_embedding
    quant = quant.reshape(b, h, n, d).permute(0, 2, 1, 3).reshape(b, n, h * d)   # :1032
    out = torch.nn.functional.linear(quant, st.w_out, st.b_out)          # :1036 project_out
    if mask is not None:
        out = torch.where(mask[..., None], out, x)                         # :1044-1048
    ind = ind.reshape(b, h, n).permute(0, 2, 1)                           # :989 '1 (b h) n -> b n h'
    new_st = VQState(st.w_in, st.b_in, st.w_out, st.b_out, st.embed, st.codebook_mean, st.codebook_variance,
                     bm, bv, st.heads, st.decay)
    return out, ind, new_st, dist


def vq_codes_from_indices(st: VQState, ind: torch.Tensor) -> torch.Tensor:
    """vector_quantize.py:820-841 (shared codebook: raw embed rows, no affine)."""
    codes = st.embed[0][ind]                                              # '... h d'
    return codes.reshape(*ind.shape[:-1], -1)


# ---------------------------------------------------------------------------
# a11 / a12: unpatch + inverse transform (FE:289-310, 607-656)
# ---------------------------------------------------------------------------


def revert_patching(batch: Batch, cfg: FEConfig, per_token_loop: bool = False) -> List[torch.Tensor]:
    """FE:607-656.  per_token_loop=True mirrors the reference's Python loop
    (used only to time the CPU baseline)."""
    x = batch.patches
    z = x.shape[-1]
    p = cfg.patch_size
    images = []
    for bi in range(x.shape[0]):
        ids = batch.batched_image_ids[bi]
        pad = batch.key_pad_mask[bi]
        for image_id in ids.unique():
            sel = (ids == image_id) & ~pad
            toks = x[bi, sel]
            pos = batch.patch_positions[bi, sel]
            chs = batch.patch_channels[bi, sel]
            ph, pw = batch.patch_sizes[len(images)]
            img = torch.zeros(cfg.channels, ph, pw, z, dtype=x.dtype)
            if per_token_loop:
                for t, ps, c in zip(toks, pos, chs):
                    img[c, ps[0], ps[1], :] = t
            else:
                img[chs, pos[:, 0], pos[:, 1]] = toks
            img = img.view(cfg.channels, ph, pw, p, p).permute(0, 1, 3, 2, 4).reshape(cfg.channels, ph * p, pw * p)
            images.append(img)
    return images


def postprocess(batch: Batch, cfg: FEConfig, per_token_loop: bool = False) -> List[torch.Tensor]:
    """FE:289-310"""
    out = []
    for img, (h, w) in zip(revert_patching(batch, cfg, per_token_loop), batch.original_sizes):
        full = torch.zeros(cfg.channels, h, w, dtype=img.dtype)
        full[:, : img.shape[1], : img.shape[2]] = img
        out.append(transform_image_out(full))
    return out


# ---------------------------------------------------------------------------
# composed paths used by the tests and the CPU baseline
# ---------------------------------------------------------------------------


def encode(images: Sequence[torch.Tensor], cfg: FEConfig, tables: NormTables, lcfg: LFQConfig,
           batch_size: Optional[int] = None, rng=random, stable: bool = True,
           build_attn_mask: bool = False):
    """preprocess -> iter_batches -> PatchNorm(eval) -> LFQ(eval).

    Returns a list of (Batch with normalised patches, indices)."""
    items = [preprocess(im, cfg, rng, stable) for im in images]
    loader = [{k: [it[k] for it in items] for k in items[0]}]
    outs = []
    for batch in iter_batches(iter(loader), cfg, batch_size, build_attn_mask):
        y = norm_forward_eval(tables, batch.patches, batch.patch_channels, batch.h_indices, batch.w_indices)
        _, idx = lfq_forward(y, lcfg)
        batch.patches = y
        outs.append((batch, idx))
    return outs
