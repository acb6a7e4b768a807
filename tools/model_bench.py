#!/usr/bin/env python3
"""Throughput of the DCTAutoencoder forward on MI355X:
the reference's patch14-l configuration (conf/patch14-l.json: hidden 1024,
16 heads, MLP 4096, 8 + 8 layers, LFQ 16 x 2^13), random init, R packed rows
of S = 3072 synthetic tokens (one 512x512 image per row, no padding).
Reports ms per forward, tokens/s, and per-kernel TFLOP/s against the dense
bf16 MFMA peak (2.5 PFLOP/s).

    python tools/model_bench.py [--rows R] [--steps K]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BF16_PEAK_TF = 2500.0


def model_flops(r, s, d=1024, inter=4096, layers=8, ncb=16, cbd=13, pp=196):
    m = r * s
    lin_layer = 2 * m * d * (3 * d + d + 2 * inter)
    attn_layer = 4 * r * s * s * d
    lin = 2 * layers * lin_layer + 2 * m * pp * d + 2 * m * d * ncb * cbd * 2 + 2 * m * d * pp
    return lin, 2 * layers * attn_layer


def run(rows=4, steps=5, warmup=2, dev=None):
    import _pkgload
    pkg = _pkgload.load()
    dev = dev or torch.device("cuda", 0)
    torch.manual_seed(0)
    enc = dict(hidden_size=1024, intermediate_size=4096, num_attention_heads=16, num_hidden_layers=8)
    cfg = pkg.DCTAutoencoderConfig(image_channels=3, patch_size=14, max_patch_h=32, max_patch_w=32,
                                   vq_codebook_size=8192, vq_num_codebooks=16, vq_type="lfq",
                                   encoder_config=enc, decoder_config=enc)
    m = pkg.DCTAutoencoder(cfg).to(dev).eval()
    s = 3072
    g = torch.Generator(device="cpu").manual_seed(1)
    patches = torch.randn(rows, s, 196, generator=g).clamp(-6, 6).to(dev)
    pos = torch.stack(torch.meshgrid(torch.arange(32), torch.arange(32), indexing="ij"), -1).reshape(-1, 2)
    pos = pos.repeat_interleave(3, 0)[None].expand(rows, s, 2).contiguous().to(dev)
    ch = torch.arange(3).repeat(1024)[None].expand(rows, s).contiguous().to(dev)

    def batch():
        return pkg.DCTPatches(patches=patches.clone(), key_pad_mask=torch.zeros(rows, s, dtype=torch.bool, device=dev),
                              batched_image_ids=torch.zeros(rows, s, dtype=torch.long, device=dev),
                              patch_channels=ch, patch_positions=pos, patch_sizes=[(36, 36)] * rows,
                              original_sizes=[(512, 512)] * rows)

    from importlib import import_module
    L = import_module("dct_autoencoder_amd._lib")
    ctx = L.context(dev)
    for _ in range(warmup):
        m(batch())
    torch.cuda.synchronize(dev)
    ctx.lib.dctae_timing_reset(ctx.h)
    ctx.lib.dctae_set_timing(ctx.h, 1)
    bs = [batch() for _ in range(steps)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for b in bs:
        m(b)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ctx.lib.dctae_set_timing(ctx.h, 0)
    ctx.lib.dctae_timing_collect(ctx.h)
    import ctypes as C
    kern, i = {}, 0
    while True:
        name, ms, n = C.c_char_p(), C.c_double(), C.c_int64()
        if ctx.lib.dctae_timing_get(ctx.h, i, C.byref(name), C.byref(ms), C.byref(n)) != 0:
            break
        kern[name.value.decode()] = {"total_ms_per_forward": round(ms.value / steps, 4), "launches": int(n.value)}
        i += 1
    lin_f, attn_f = model_flops(rows, s)
    out = {"workload": f"DCTAutoencoder forward (encode + LFQ + decode), patch14-l, {rows} rows x {s} tokens, bf16 "
                       f"MFMA, fp32 accumulate / residual", "ms_per_forward": round(el / steps * 1e3, 3),
           "tokens_per_s": round(rows * s * steps / el, 1), "total_tflops": round((lin_f + attn_f) * steps / el / 1e12, 1),
           "kernels": kern}
    if "model_linear" in kern:
        t = kern["model_linear"]["total_ms_per_forward"] / 1e3
        out["linear"] = {"achieved_tflops": round(lin_f / t / 1e12, 1), "peak": BF16_PEAK_TF,
                         "frac": round(lin_f / t / 1e12 / BF16_PEAK_TF, 4)}
    if "model_attention" in kern:
        t = kern["model_attention"]["total_ms_per_forward"] / 1e3
        out["attention"] = {"achieved_tflops": round(attn_f / t / 1e12, 1), "peak": BF16_PEAK_TF,
                            "frac": round(attn_f / t / 1e12 / BF16_PEAK_TF, 4)}
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    print(json.dumps(run(a.rows, a.steps)))
