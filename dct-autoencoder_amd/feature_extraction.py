"""DCTAutoencoderFeatureExtractor — drop-in for the reference's
dct_autoencoder/feature_extraction_dct_autoencoder.py:107-656 (FE below),
running on MI355X through libdctae.

Reference methods keep their names, arguments and results:
  preprocess(im)                 FE:154-177   -> dict(patches, positions, channels, original_sizes, patch_sizes)
  iter_batches(loader, bs)       FE:179-287   -> DCTPatches generator (same emission quirks)
  postprocess(dct_patches)       FE:289-310   -> list of (3, H, W) RGB images
  revert_patching(dct_patches)   FE:607-656   -> list of (3, 14ph, 14pw) spectra
  _transform_image_in / _transform_image_out   FE:129-152 (dctae_dct2)
  _get_crop_dims / _crop_image / _patch_image (dctae_patch_spectrum) / _group_patches_by_max_seq_len / _batch_groups
Stage hooks: callers replace these per instance or in a subclass (the
reference's decode_gif.py:86-91 sets ``_transform_image_out = lambda x: x`` to
render the spectrum; its tests/testpatching.py:42-43 makes both transforms the
identity).  preprocess / postprocess / iter_batches / encode_batch then run the
reference's stage sequence (FE:154-177, 179-287, 289-310) through the hooks,
each default stage still a HIP kernel; with no override they run the fused
launch sequence.
Additive fused entry points (the MI355X hot path):
  encode_batch(images, patchnorm, lfq, batch_size)  preprocess + pack + PatchNorm + LFQ in one launch sequence
  decode_batch(dct_patches, codes, patchnorm, lfq)  indices_to_codes + inverse_norm + postprocess

Deviations (documented in DESIGN.md):
  * tokens of equal importance score are ordered by flat index (the
    reference's CPU sort is unstable at ties, FE:418);
  * everything stays on the input's HIP device (the reference round-trips
    through the CPU for the FFT, FE:138-141, and keeps batches on the CPU,
    FE:204-207);
  * ``DCTPatches.attn_mask`` is computed lazily.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass
from typing import Any, Dict, Iterator, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from . import _ops, packing
from ._ops import FEParams
from .dct_patches import DCTPatches


@dataclass
class GroupPatchesState:
    """FE:96-104"""
    groups: List[List[torch.Tensor]]
    groups_pos: List[List[torch.Tensor]]
    group: List[torch.Tensor]
    group_pos: List[torch.Tensor]
    groups_channels: List[List[torch.Tensor]]
    group_channels: List[torch.Tensor]
    seq_len: int


class DCTAutoencoderFeatureExtractor:
    def __init__(self, channels: int, patch_size: int, sample_patches_beta: float, max_patch_h: int,
                 max_patch_w: int, max_seq_len: int, channel_importances: Tuple[float, float, float] = (8.0, 1.0, 1.0),
                 patch_sample_magnitude_weight: float = 0.1, device=None):
        self.channels = channels
        self.patch_size = patch_size
        self.sample_patches_beta = sample_patches_beta
        self.max_patch_h = max_patch_h
        self.max_patch_w = max_patch_w
        self.max_seq_len = max_seq_len
        self.channel_importances = torch.Tensor(channel_importances)
        self.patch_sample_magnitude_weight = patch_sample_magnitude_weight
        self.device = device
        self.rng = random  # python ``random`` stream used for k ~ Exp(beta) (util.py:171)

    # ------------------------------------------------------------------ helpers
    def params(self, max_seq_len: Optional[int] = None) -> FEParams:
        return FEParams(channels=self.channels, patch_size=self.patch_size, max_patch_h=self.max_patch_h,
                        max_patch_w=self.max_patch_w,
                        max_seq_len=self.max_seq_len if max_seq_len is None else max_seq_len,
                        channel_importances=tuple(float(v) for v in self.channel_importances.tolist()),
                        magnitude_weight=float(self.patch_sample_magnitude_weight))

    def _dev(self, t: torch.Tensor) -> torch.Tensor:
        if t.is_cuda:
            return t
        if not torch.cuda.is_available():
            from ._lib import DCTAEUnavailable
            raise DCTAEUnavailable("no HIP device: the MI355X path has no CPU fallback")
        dev = self.device if self.device is not None else torch.device("cuda", torch.cuda.current_device())
        return t.to(dev)

    def _tokens(self, h: int, w: int) -> int:
        return packing.tokens_per_image(h, w, self.channels, self.patch_size, self.max_patch_h, self.max_patch_w)

    def _k(self, h: int, w: int) -> int:
        return packing.choose_k(self._tokens(h, w), self.sample_patches_beta, self.max_seq_len, self.rng)

    # ------------------------------------------------------------- stage hooks
    def _overridden(self, name: str) -> bool:
        """True when a caller replaced the stage `name` on this instance or in a subclass."""
        return name in self.__dict__ or getattr(type(self), name) is not getattr(DCTAutoencoderFeatureExtractor, name)

    def _staged_in(self) -> bool:
        return any(self._overridden(n) for n in ("_transform_image_in", "_crop_image", "_patch_image"))

    def _staged_out(self) -> bool:
        return any(self._overridden(n) for n in ("_transform_image_out", "revert_patching"))

    @torch.no_grad()
    def _transform_image_in(self, x: torch.Tensor) -> torch.Tensor:
        """FE:129-142: rgb_to_ipt, then the orthonormal dct2 of the whole
        (c, h, w) image (dctae_dct2); result in x's dtype and on x's device.
        The reference runs rgb_to_ipt in the input's dtype before ``.float()``:
        fp16 / bf16 inputs get that arithmetic (dctae_dct2 color 2 / 3)."""
        color = {torch.float16: 2, torch.bfloat16: 3}.get(x.dtype, 1)
        y = _ops.dct2(self._dev(x).float(), inverse=False, color=color)
        return y.to(x.dtype).to(x.device)

    def _transform_image_out(self, x: torch.Tensor) -> torch.Tensor:
        """FE:144-152: idct2 of the whole (c, h, w) spectrum, then ipt_to_rgb (dctae_dct2)."""
        y = _ops.dct2(self._dev(x).float(), inverse=True, color=True)
        return y.to(x.dtype).to(x.device)

    # ------------------------------------------------------------- reference API
    def _get_crop_dims(self, h: int, w: int):
        """FE:312-345"""
        return packing.crop_dims(h, w, self.patch_size)

    @torch.no_grad()
    def _crop_image(self, x: torch.Tensor) -> torch.Tensor:
        """FE:347-362"""
        c, h, w = x.shape
        assert c == self.channels
        ch, cw = self._get_crop_dims(h, w)
        return x[:, :ch, :cw]

    @torch.no_grad()
    def _patch_image(self, x: torch.Tensor):
        """FE:364-452 on a cropped (c, h, w) spectrum (dctae_patch_spectrum):
        tiles of the kept corner, importance order (score desc, flat index asc),
        top k (k drawn like the reference, FE:429-435)."""
        c, h, w = x.shape
        P = self.patch_size
        assert h % P == 0
        assert w % P == 0
        assert c == self.channels
        k = self._k(h, w)
        patches, pos, channels = _ops.patch_spectrum(self._dev(x), self.params(), k)
        patches = patches.to(x.dtype)   # the reference's patches keep the spectrum's dtype
        s, z = patches.shape
        assert z == P ** 2, f"{z} != {P ** 2}"
        assert s <= self.max_seq_len
        return patches, pos, channels

    @torch.no_grad()
    def preprocess(self, im: torch.Tensor) -> Dict[str, Any]:
        """FE:154-177 for one (c, h, w) RGB image in [0, 1]: IPT + DCT +
        spectral patching + importance order + top-k, all on the GPU.  With
        an overridden stage hook the reference's stage sequence runs instead."""
        if self._staged_in():
            return self._preprocess_staged(im)
        return self.preprocess_many([im])[0]

    @torch.no_grad()
    def _preprocess_staged(self, im: torch.Tensor) -> Dict[str, Any]:
        """FE:154-177 stage by stage, every stage through its (possibly replaced) hook."""
        im = self._transform_image_in(im)
        _, h, w = im.shape
        original_size = (h, w)
        im = self._crop_image(im)
        _, ch, cw = im.shape
        patch_size = (ch // self.patch_size, cw // self.patch_size)
        patches, pos, channels = self._patch_image(im)
        return dict(patches=patches, positions=pos, channels=channels, original_sizes=original_size,
                    patch_sizes=patch_size)

    @torch.no_grad()
    def preprocess_many(self, images: Sequence[torch.Tensor]) -> List[Dict[str, Any]]:
        """``preprocess`` for several images in one launch sequence."""
        if self._staged_in() or any(im.dtype != torch.float32 for im in images):
            # fp16 / bf16 images: the reference's stage sequence, whose colour
            # transform runs in the input dtype (FE:135-141)
            return [self._preprocess_staged(im) for im in images]
        images = [self._dev(im) for im in images]
        for im in images:
            assert im.shape[0] == self.channels
        ks = [self._k(im.shape[1], im.shape[2]) for im in images]
        S = max(ks)
        rows = [[i] for i in range(len(images))]
        plan = packing.layout(rows, dict(enumerate(ks)))
        desc, dev, keep = _ops.image_set(images)
        res = _ops.encode(desc, dev, self.params(S), plan, len(images), S, None, None, want_codes=False,
                          want_raw=True)
        out = []
        for i, im in enumerate(images):
            k = ks[i]
            h, w = im.shape[1], im.shape[2]
            out.append(dict(patches=res["raw"][i, :k], positions=res["positions"][i, :k],
                            channels=res["channels"][i, :k], original_sizes=(h, w),
                            patch_sizes=packing.patch_grid(h, w, self.patch_size)))
        return out

    @torch.no_grad()
    def iter_batches(self, dataloader, batch_size: Optional[int] = None) -> Iterator[DCTPatches]:
        """FE:179-287: greedy packing of preprocessed items into rows of
        max_seq_len; same emission rules (see packing.iter_batch_plans)."""
        if self._overridden("_group_patches_by_max_seq_len"):
            yield from self._iter_batches_staged(dataloader, batch_size)
            return
        fixed = {"patches", "positions", "channels", "original_sizes", "patch_sizes"}
        items: Dict[int, Tuple] = {}
        cum_o: List = []
        cum_p: List = []
        cum_x: Dict[str, List] = {}
        st = None
        nxt = 0
        max_tok = self.max_patch_h * self.max_patch_w * self.channels
        while True:
            try:
                d = next(dataloader)
            except StopIteration:
                return
            ids = list(range(nxt, nxt + len(d["patches"])))
            nxt += len(ids)
            for i, pt, ps, ch in zip(ids, d["patches"], d["positions"], d["channels"]):
                items[i] = (pt, ps, ch)
            cum_o = cum_o + list(d["original_sizes"])
            cum_p = cum_p + list(d["patch_sizes"])
            for k, v in d.items():
                if k not in fixed:
                    cum_x.setdefault(k, []).extend(v)
            st = packing.group([items[i][0].shape[0] for i in ids], ids, self.max_seq_len, max_tok, st)
            if batch_size is None and st.cur:
                st.rows.append(st.cur)
                st.cur, st.seq_len = [], 0
            if batch_size is None or len(st.rows) > batch_size:
                emit = st.rows[:batch_size]
                st = packing.GroupState(rows=st.rows[batch_size:], cur=st.cur, seq_len=st.seq_len)
                n = sum(len(r) for r in emit)
                o_now, cum_o = cum_o[:n], cum_o[n:]
                p_now, cum_p = cum_p[:n], cum_p[n:]
                x_now = {k: v[:n] for k, v in cum_x.items()}
                cum_x = {k: v[n:] for k, v in cum_x.items()}
                batch = self._batch_groups([[items[i][0] for i in r] for r in emit],
                                           [[items[i][1] for i in r] for r in emit],
                                           [[items[i][2] for i in r] for r in emit],
                                           original_sizes=o_now, patch_sizes=p_now, _data=x_now)
                if batch_size is not None:
                    assert batch.patches.shape[0] == batch_size
                    # emitted groups leave the state for good (FE:235-243): drop their items
                    for r in emit:
                        for i in r:
                            items.pop(i, None)
                yield batch

    @torch.no_grad()
    def _iter_batches_staged(self, dataloader, batch_size: Optional[int]) -> Iterator[DCTPatches]:
        """FE:179-287 step by step through the (replaced) _group_patches_by_max_seq_len
        and _batch_groups hooks."""
        fixed = {"patches", "positions", "channels", "original_sizes", "patch_sizes"}
        state = None
        cum_o, cum_p, cum_x = [], [], {}
        while True:
            try:
                d = next(dataloader)
            except StopIteration:
                return
            cum_o = cum_o + list(d["original_sizes"])
            cum_p = cum_p + list(d["patch_sizes"])
            for k, v in d.items():
                if k not in fixed:
                    cum_x.setdefault(k, []).extend(v)
            state = self._group_patches_by_max_seq_len(d["patches"], d["positions"], d["channels"], state)
            if batch_size is None and len(state.group) > 0:
                state.groups.append(state.group)
                state.groups_pos.append(state.group_pos)
                state.groups_channels.append(state.group_channels)
                state.seq_len, state.group, state.group_pos, state.group_channels = 0, [], [], []
            if batch_size is None or len(state.groups) > batch_size:
                keep = GroupPatchesState(state.groups[batch_size:], state.groups_pos[batch_size:], state.group,
                                         state.group_pos, state.groups_channels[batch_size:], state.group_channels,
                                         state.seq_len)
                emit = (state.groups[:batch_size], state.groups_pos[:batch_size], state.groups_channels[:batch_size])
                n = sum(len(g) for g in emit[0])
                batch = self._batch_groups(*emit, original_sizes=cum_o[:n], patch_sizes=cum_p[:n],
                                           _data={k: v[:n] for k, v in cum_x.items()})
                if batch_size is not None:
                    assert batch.patches.shape[0] == batch_size
                cum_o, cum_p = cum_o[n:], cum_p[n:]
                cum_x = {k: v[n:] for k, v in cum_x.items()}
                state = keep
                yield batch

    @torch.no_grad()
    def _group_patches_by_max_seq_len(self, batched_patches, batched_positions, batched_channels, state=None):
        """FE:454-513 (kept for callers that drive the grouping themselves)."""
        if state is None:
            state = GroupPatchesState([], [], [], [], [], [], 0)
        for patches, pos, channels in zip(batched_patches, batched_positions, batched_channels):
            k = patches.shape[0]
            assert k <= self.max_patch_h * self.max_patch_w * self.channels and k <= self.max_seq_len, \
                f"patch with len {k} exceeds maximum sequence length"
            assert k == channels.shape[0]
            if state.seq_len + k > self.max_seq_len:
                state.groups.append(state.group)
                state.groups_pos.append(state.group_pos)
                state.groups_channels.append(state.group_channels)
                state.group, state.group_pos, state.group_channels, state.seq_len = [], [], [], 0
            state.group.append(patches)
            state.group_pos.append(pos)
            state.group_channels.append(channels)
            state.seq_len += k
        return state

    @torch.no_grad()
    def _batch_groups(self, grouped_batched_patches, grouped_batched_positions, grouped_batched_channels,
                      device=None, **dct_patch_kwargs) -> DCTPatches:
        """FE:515-605: concatenate rows, zero-pad to max_seq_len, image ids,
        key_pad_mask (True at padding).  attn_mask is lazy."""
        S = self.max_seq_len
        first = grouped_batched_patches[0][0]
        dev = device if device is not None else first.device
        R = len(grouped_batched_patches)
        z = first.shape[-1]
        patches = torch.zeros((R, S, z), dtype=first.dtype, device=dev)
        positions = torch.zeros((R, S, 2), dtype=torch.long, device=dev)
        channels = torch.zeros((R, S), dtype=torch.long, device=dev)
        ids = torch.zeros((R, S), dtype=torch.long, device=dev)
        lengths = []
        for r, (gp, gpos, gch) in enumerate(zip(grouped_batched_patches, grouped_batched_positions,
                                                grouped_batched_channels)):
            assert len(gp) == len(gpos) == len(gch)
            col = 0
            for j, (pt, ps, ch) in enumerate(zip(gp, gpos, gch)):
                k = pt.shape[0]
                assert pt.shape[1] == self.patch_size ** 2
                assert ps.shape[0] == k and ch.shape[0] == k
                patches[r, col:col + k] = pt
                positions[r, col:col + k] = ps
                channels[r, col:col + k] = ch
                ids[r, col:col + k] = j
                col += k
            assert col <= S
            lengths.append(col)
        lengths = torch.tensor(lengths, dtype=torch.long, device=dev)
        key_pad_mask = lengths[:, None] <= torch.arange(S, device=dev)[None, :]
        return DCTPatches(patches=patches, key_pad_mask=key_pad_mask, attn_mask=None, batched_image_ids=ids,
                          patch_positions=positions, patch_channels=channels, **dct_patch_kwargs)

    @torch.no_grad()
    def revert_patching(self, output: DCTPatches) -> List[torch.Tensor]:
        """FE:607-656: per image a zero (c, 14ph, 14pw) spectrum holding its tokens."""
        x = output.patches
        p = self.patch_size
        ids = output.batched_image_ids
        pad = output.key_pad_mask
        images = []
        for bi in range(x.shape[0]):
            for image_id in torch.unique(ids[bi]).tolist():
                sel = (ids[bi] == image_id) & ~pad[bi]
                ph, pw = output.patch_sizes[len(images)]
                img = torch.zeros(self.channels, ph, pw, x.shape[-1], dtype=x.dtype, device=x.device)
                pos = output.patch_positions[bi, sel]
                img[output.patch_channels[bi, sel], pos[:, 0], pos[:, 1]] = x[bi, sel]
                img = img.view(self.channels, ph, pw, p, p).permute(0, 1, 3, 2, 4).reshape(self.channels, ph * p, pw * p)
                images.append(img)
        return images

    @torch.no_grad()
    def postprocess(self, x: DCTPatches) -> List[torch.Tensor]:
        """FE:289-310: un-normalised DCTPatches -> RGB images (revert_patching,
        zero pad, DCT-III, IPT -> RGB fused on the GPU).  With an overridden
        _transform_image_out / revert_patching the reference's stage sequence
        runs through the hooks (e.g. the spectrum itself for decode_gif.py:86-91)."""
        if self._staged_out():
            images = []
            for image, (h, w) in zip(self.revert_patching(x), x.original_sizes):
                ch, cw = image.shape[-2:]
                im_pad = torch.zeros(self.channels, h, w, device=image.device, dtype=image.dtype)
                im_pad[:, :ch, :cw] = image
                images.append(self._transform_image_out(im_pad))
            return images
        return _ops.decode(self.params(x.patches.shape[1]), x.batched_image_ids, x.key_pad_mask,
                           x.patch_positions, x.patch_channels, x.patch_sizes, x.original_sizes,
                           patches=x.patches)

    # ------------------------------------------------------- fused MI355X path
    @torch.no_grad()
    def encode_batch(self, images, patchnorm=None, lfq=None, batch_size: Optional[int] = None,
                     return_patches: bool = False, return_raw: bool = False, return_scores: bool = False,
                     ks: Optional[Sequence[int]] = None) -> List[Tuple[DCTPatches, Optional[torch.Tensor]]]:
        """preprocess every image, pack (iter_batches over ONE dataloader item
        holding all images, FE:179-287), PatchNorm (eval) and LFQ — the
        encode half of SURVEY §3.1-3.3 — in one launch sequence per batch.

        images: (B, 3, H, W) tensor or a list of (3, H, W) tensors on the GPU.
        Returns [(DCTPatches, codes)] per emitted batch; DCTPatches.patches
        holds the PatchNorm output if return_patches, the raw DCT tokens if
        return_raw, else an empty (R, S, 0) tensor.  codes is None without lfq.
        With an overridden stage hook the reference's stages run one by one.
        """
        if self._staged_in() or self._overridden("_group_patches_by_max_seq_len") or \
                self._overridden("_batch_groups"):
            return self._encode_staged(images, patchnorm, lfq, batch_size, return_patches, return_raw)
        if isinstance(images, torch.Tensor) and images.dim() == 4:
            x = self._dev(images)
            B, _, H, W = x.shape
            sizes = [(H, W)] * B
            desc, dev, keep = _ops.batch_image_set(x)
            img_list = None
        else:
            img_list = [self._dev(im) for im in images]
            sizes = [(im.shape[1], im.shape[2]) for im in img_list]
            desc, dev, keep = _ops.image_set(img_list)
        if ks is None:
            ks = [self._k(h, w) for h, w in sizes]
        max_tok = self.max_patch_h * self.max_patch_w * self.channels
        plans = list(packing.iter_batch_plans([(ks, list(range(len(ks))))], self.max_seq_len, max_tok, batch_size))
        if lfq is not None and patchnorm is None:
            raise AssertionError("LFQ codes need a PatchNorm")
        # LFQ with projections (dim != codebook_dim * num_codebooks, lfq.py:54-62,
        # e.g. conf/patch14-l.json's 196 -> 16 x 13): the fused launch stops at the
        # PatchNorm output and the fused project_in + sign + pack kernel
        # (dctae_lfq_project_in) follows on the same stream
        proj = lfq is not None and lfq.has_projections
        want_norm = return_patches or proj
        norm = patchnorm.state(thresholds=not want_norm) if patchnorm is not None else None
        lcfg = lfq.cfg() if lfq is not None and not proj else None
        outs = []
        for rows in plans:
            plan = packing.layout(rows, dict(enumerate(ks)))
            sub = self._subset(desc, keep, plan.images) if len(plan.images) != len(ks) else desc
            plan_local = packing.layout([[plan.images.index(i) for i in r] for r in rows],
                                        {j: ks[i] for j, i in enumerate(plan.images)}) \
                if len(plan.images) != len(ks) else plan
            res = _ops.encode(sub, dev, self.params(), plan_local, plan.n_rows, self.max_seq_len, norm, lcfg,
                              want_codes=lcfg is not None, want_patches=want_norm, want_raw=return_raw,
                              want_scores=return_scores)
            if proj:   # codes only: lfq.py:136-187 without the quantized output's project_out
                # fused project_in + sign + pack on the PatchNorm output, whose clamp
                # (patchnorm.py:163) bounds it: the kernels of BatchEncoder's staged path
                xb = max(abs(norm.min_val), abs(norm.max_val))
                res["codes"] = lfq.project_codes(res["patches"], x_bound=xb if 0.0 < xb < math.inf else None)
            pt = res["patches"] if return_patches else res.get("raw")
            if pt is None:
                pt = torch.empty((plan.n_rows, self.max_seq_len, 0), device=dev)
            dp = DCTPatches(patches=pt, key_pad_mask=res["key_pad_mask"], attn_mask=None,
                            batched_image_ids=res["image_ids"], patch_channels=res["channels"],
                            patch_positions=res["positions"],
                            patch_sizes=[packing.patch_grid(*sizes[i], self.patch_size) for i in plan.images],
                            original_sizes=[tuple(sizes[i]) for i in plan.images])
            if return_patches and return_raw:
                dp._data = {"raw_patches": res["raw"]}
            if return_scores:
                dp._data = (dp._data or {}) | {"scores": res["scores"]}
            outs.append((dp, res.get("codes")))
        return outs

    @torch.no_grad()
    def _encode_staged(self, images, patchnorm, lfq, batch_size, return_patches, return_raw):
        """encode_batch through the stage hooks: preprocess -> iter_batches ->
        PatchNorm (eval) -> LFQ (eval), each stage on its own launch."""
        items = [self.preprocess(im) for im in images]
        loader = iter([{k: [it[k] for it in items] for k in items[0]}])
        outs = []
        for batch in self.iter_batches(loader, batch_size):
            codes, normed = None, None
            if patchnorm is not None:
                normed = patchnorm(batch.shallow_copy())
                if lfq is not None:
                    _, codes, _, _ = lfq(normed, mask=~batch.key_pad_mask)
            if not return_raw:
                batch.patches = normed if (return_patches and normed is not None) else \
                    torch.empty((*batch.patches.shape[:2], 0), device=batch.patches.device)
            elif return_patches and normed is not None:
                batch._data = (batch._data or {}) | {"normalised_patches": normed}
            outs.append((batch, codes))
        return outs

    @staticmethod
    def _subset(desc, keep, idx):
        import ctypes as C
        from ._lib import Images, i32, i64
        offs = [keep[1][i] for i in idx]
        hw = []
        for i in idx:
            hw += [keep[2][2 * i], keep[2][2 * i + 1]]
        k2 = [i64(offs), i32(hw)]
        keep.append(k2)
        return Images(desc.rgb_dev, C.cast(k2[0], C.POINTER(C.c_int64)), C.cast(k2[1], C.POINTER(C.c_int32)), len(idx))

    @torch.no_grad()
    def decode_batch(self, dct_patches: DCTPatches, codes: torch.Tensor, patchnorm, lfq) -> List[torch.Tensor]:
        """LFQ.indices_to_codes -> PatchNorm.inverse_norm -> postprocess, fused
        (the decode half of SURVEY §3.4 without the transformer).  With LFQ
        projections the codes go through the fused codes -> project_out kernel and the HIP
        inverse PatchNorm first, and the fused decode starts from the tokens."""
        staged = self._staged_out()   # an overridden revert_patching / _transform_image_out (FE:289-310)
        if lfq.has_projections or staged:
            dp = dct_patches.shallow_copy()
            if lfq.has_projections and lfq._fused_proj() and lfq.dim == self.patch_size ** 2 and not staged:
                # project_out alone, the inverse PatchNorm inside the decode
                # (dctae_decode_normed)
                w, b = lfq._proj_w(lfq.project_out, codes.device)
                x = _ops.lfq_project_out(codes, w, b, lfq.cfg())
                return _ops.decode(self.params(dp.key_pad_mask.shape[1]), dp.batched_image_ids, dp.key_pad_mask,
                                   dp.patch_positions, dp.patch_channels, dp.patch_sizes, dp.original_sizes,
                                   patches=x, norm=patchnorm.state(thresholds=False), normed=True)
            else:
                dp.patches = lfq.indices_to_codes(codes)
                dp.patches = patchnorm.inverse_norm(dp)
            return self.postprocess(dp)
        return _ops.decode(self.params(dct_patches.key_pad_mask.shape[1]), dct_patches.batched_image_ids,
                           dct_patches.key_pad_mask, dct_patches.patch_positions, dct_patches.patch_channels,
                           dct_patches.patch_sizes, dct_patches.original_sizes, codes=codes,
                           norm=patchnorm.state(), lfq=lfq.cfg())


class BatchEncoder:
    """Pre-planned fused encode for a fixed batch geometry (the bench and
    serving path): packing plan, ctypes descriptors and output buffers are
    built once; each call only enqueues the kernels (dctae_encode)."""

    def __init__(self, fe: DCTAutoencoderFeatureExtractor, batch: int, height: int, width: int, patchnorm, lfq,
                 device=None, want_patches: bool = False):
        import ctypes as C
        from ._lib import Images, LFQCfg, Packing, PackedOut, i32, i64, ptr
        self.fe = fe
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.dev.index is None:   # "cuda" -> the current device, as tensors report it
            self.dev = torch.device(self.dev.type, torch.cuda.current_device())
        self.B, self.H, self.W = batch, height, width
        if fe.sample_patches_beta > 0:
            raise AssertionError("BatchEncoder needs sample_patches_beta == 0 (fixed k)")
        k = fe._tokens(height, width)
        k = min(k, fe.max_seq_len)
        max_tok = fe.max_patch_h * fe.max_patch_w * fe.channels
        (rows,) = list(packing.iter_batch_plans([([k] * batch, list(range(batch)))], fe.max_seq_len, max_tok, None))
        self.plan = packing.layout(rows, {i: k for i in range(batch)})
        self.k = k
        self.n_rows = self.plan.n_rows
        self.S = fe.max_seq_len
        # LFQ with projections (lfq.py:54-62): with every packed row full,
        # dctae_encode_lfq_proj runs project_in + sign + pack on the staged
        # PatchNorm output before the sort / pack; otherwise the fused launch
        # stops at the packed PatchNorm output and dctae_lfq_project_in follows
        self.lfq = lfq
        self.proj = lfq.has_projections
        if self.proj and not lfq._fused_proj():
            raise NotImplementedError("BatchEncoder: LFQ projections of this shape run through encode_batch")
        self.proj_staged = (self.proj and all(n == fe.max_seq_len for n in self.plan.row_len)
                            and lfq.codebook_dim <= 16 and (fe.patch_size ** 2) % 4 == 0)
        want_norm = want_patches or (self.proj and not self.proj_staged)
        self.norm = patchnorm.state(thresholds=not want_norm)
        self.lcfg = lfq.cfg()
        self.p = fe.params()
        per = 3 * height * width
        self._keep = [i64([i * per for i in range(batch)]), i32([height, width] * batch)]
        pl = self.plan
        self._pk_keep = [i32(pl.row), i32(pl.col), i32(pl.k), i32(pl.local_id), i32(pl.row_len)]
        self.packing = Packing(*[C.cast(a, C.POINTER(C.c_int32)) for a in self._pk_keep], self.n_rows)
        R, S = self.n_rows, self.S
        self.out = {
            "codes": torch.empty((R, S, self.lcfg.num_codebooks), dtype=torch.long, device=self.dev),
            "positions": torch.empty((R, S, 2), dtype=torch.long, device=self.dev),
            "channels": torch.empty((R, S), dtype=torch.long, device=self.dev),
            "image_ids": torch.empty((R, S), dtype=torch.long, device=self.dev),
            "key_pad_mask": torch.empty((R, S), dtype=torch.bool, device=self.dev),
        }
        if want_norm:
            self.out["patches"] = torch.empty((R, S, fe.patch_size ** 2), dtype=torch.float32, device=self.dev)
        o = self.out
        self.po = PackedOut(ptr(None if self.proj and not self.proj_staged else o["codes"]), ptr(o["positions"]), ptr(o["channels"]), ptr(o["image_ids"]),
                            ptr(o["key_pad_mask"]), ptr(o.get("patches")), None, None)
        self._ncfg = self.norm.c()
        self._cfg = self.p.c(S)
        from . import _lib
        self.ctx = _lib.context(self.dev)

    def __call__(self, x: torch.Tensor):
        import ctypes as C
        from ._lib import Images, ptr, stream_ptr
        assert x.shape == (self.B, 3, self.H, self.W) and x.dtype == torch.float32 and x.is_contiguous()
        assert x.device == self.dev
        imgs = Images(C.c_void_p(x.data_ptr()), C.cast(self._keep[0], C.POINTER(C.c_int64)),
                      C.cast(self._keep[1], C.POINTER(C.c_int32)), self.B)
        if self.proj_staged:
            w, b = self.lfq._proj_w(self.lfq.project_in, self.dev)
            rc = self.ctx.lib.dctae_encode_lfq_proj(self.ctx.h, C.byref(self._cfg), C.byref(imgs),
                                                    C.byref(self.packing), C.byref(self._ncfg), C.byref(self.lcfg),
                                                    ptr(w), ptr(b), C.byref(self.po), stream_ptr(self.dev))
            self.ctx.check(rc, "dctae_encode_lfq_proj")
            return self.out
        rc = self.ctx.lib.dctae_encode(self.ctx.h, C.byref(self._cfg), C.byref(imgs), C.byref(self.packing),
                                       C.byref(self._ncfg), None if self.proj else C.byref(self.lcfg),
                                       C.byref(self.po), stream_ptr(self.dev))
        self.ctx.check(rc, "dctae_encode")
        if self.proj:
            w, b = self.lfq._proj_w(self.lfq.project_in, self.dev)
            from . import _ops
            self.out["codes"] = _ops.lfq_project_in_into(self.out["patches"], w, b, self.lcfg, self.out["codes"])
        return self.out


class BatchDecoder:
    """Pre-planned fused decode for a BatchEncoder's fixed geometry (config 3
    round trip): LFQ.indices_to_codes -> PatchNorm.inverse_norm ->
    revert_patching -> IDCT -> IPT -> RGB of the encoder's packed outputs
    (dctae_decode), images in the reference's enumeration order (rows in
    order, image ids ascending, FE:619-633) into one (B, 3, H, W) tensor."""

    def __init__(self, enc: "BatchEncoder", patchnorm, lfq):
        import ctypes as C
        from ._lib import i32, i64
        self.enc = enc
        pl = enc.plan
        order = sorted(range(enc.B), key=lambda i: (pl.row[i], pl.local_id[i]))
        self.lut_w = max(pl.local_id) + 1
        lut = [-1] * (enc.n_rows * self.lut_w)
        for n, i in enumerate(order):
            lut[pl.row[i] * self.lut_w + pl.local_id[i]] = n
        H, W, p = enc.H, enc.W, enc.fe.patch_size
        per = 3 * H * W
        self._keep = [i32(lut), i32([H, W] * enc.B), i64([n * per for n in range(enc.B)]),
                      i32([H // p, W // p] * enc.B)]
        self._ptr = [C.cast(self._keep[0], C.POINTER(C.c_int32)), C.cast(self._keep[1], C.POINTER(C.c_int32)),
                     C.cast(self._keep[2], C.POINTER(C.c_int64)), C.cast(self._keep[3], C.POINTER(C.c_int32))]
        self.norm = patchnorm.state(thresholds=False)
        self._ncfg = self.norm.c()
        self.lcfg = lfq.cfg()
        self.lfq, self.patchnorm = lfq, patchnorm
        # LFQ with projections (lfq.py:54-62): codes -> project_out (fused MFMA
        # kernel, dctae_lfq_project_out) -> inverse PatchNorm (dctae_norm_inverse)
        # -> the fused decode from tokens
        self.proj = lfq.has_projections
        # projections: project_out alone (dctae_lfq_project_out) and the
        # inverse PatchNorm inside the decode's column kernel
        # (dctae_decode_normed: per-block (c, strip) tables instead of a
        # per-token table gather); False: project_out with the inverse fused
        # (dctae_lfq_project_out_inverse_norm) then dctae_decode
        self.normed_decode = True
        self.out = torch.empty((enc.B, 3, H, W), dtype=torch.float32, device=enc.dev)

    def __call__(self, packed) -> torch.Tensor:
        from ._lib import ptr, stream_ptr
        import ctypes as C
        e = self.enc
        lut, hw, offs, phw = self._ptr
        if self.proj:
            from . import _ops
            if self.lfq._fused_proj() and self.normed_decode:
                w, b = self.lfq._proj_w(self.lfq.project_out, e.dev)
                x = _ops.lfq_project_out(packed["codes"], w, b, self.lcfg)
                rc = e.ctx.lib.dctae_decode_normed(e.ctx.h, C.byref(e._cfg), e.n_rows, lut, self.lut_w, e.B, hw, offs,
                                                   phw, ptr(packed["image_ids"]), ptr(packed["key_pad_mask"]),
                                                   ptr(packed["positions"]), ptr(packed["channels"]),
                                                   C.byref(self._ncfg), ptr(x), ptr(self.out), stream_ptr(e.dev))
                e.ctx.check(rc, "dctae_decode_normed")
                return self.out
            if self.lfq._fused_proj():
                w, b = self.lfq._proj_w(self.lfq.project_out, e.dev)
                x = _ops.lfq_project_out_inverse_norm(packed["codes"], w, b, self.lcfg, self.norm, e.fe.params(),
                                                      packed["channels"], packed["positions"])
            else:
                x = self.lfq.indices_to_codes(packed["codes"]).float()
                x = _ops.norm_apply(x, packed["channels"], packed["positions"], self.norm, e.fe.params(),
                                    inverse=True)
            rc = e.ctx.lib.dctae_decode(e.ctx.h, C.byref(e._cfg), e.n_rows, lut, self.lut_w, e.B, hw, offs, phw,
                                        ptr(packed["image_ids"]), ptr(packed["key_pad_mask"]),
                                        ptr(packed["positions"]), ptr(packed["channels"]), None, None, None, ptr(x),
                                        ptr(self.out), stream_ptr(e.dev))
            e.ctx.check(rc, "dctae_decode")
            return self.out
        rc = e.ctx.lib.dctae_decode(e.ctx.h, C.byref(e._cfg), e.n_rows, lut, self.lut_w, e.B, hw, offs, phw,
                                    ptr(packed["image_ids"]), ptr(packed["key_pad_mask"]), ptr(packed["positions"]),
                                    ptr(packed["channels"]), C.byref(self._ncfg), C.byref(self.lcfg),
                                    ptr(packed["codes"]), None, ptr(self.out), stream_ptr(e.dev))
        e.ctx.check(rc, "dctae_decode")
        return self.out
