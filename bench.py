#!/usr/bin/env python3
"""Throughput bench of the MI355X encode hot path (BASELINE.json metric):

    Mpix/s encode (DCT + PatchNorm + LFQ), patch14, 512x512, 1/2/4/8 GPU

One step = one fused encode (dctae_encode) of a batch of B synthetic 512x512
RGB images already resident in HBM: IPT colour -> global DCT (kept 448x448
corner) -> 14x14 spectral tokens -> importance order -> packed DCTPatches
rows (S = 3072) -> PatchNorm (reference-fitted tables) -> LFQ 14 x 2^14 codes.
Multi-GPU: one process per GPU, each rank encodes its own shard (weak
scaling, no collective on the data path); time = max over ranks.  Run with
--gpus N > 1 outside torchrun, bench.py starts `python -m torch.distributed.run
--nproc-per-node N ... bench.py ...` as a CHILD process (before anything
touches the GPU) and exits with its return code; under torchrun (WORLD_SIZE
set) it is one rank.

Roofline: the metric's algorithmic bytes are 3,591,168 B per
512^2 image (fp32 RGB read + int64 codes / positions / channel / image id per
token + key_pad share).  roofline.frac = those bytes x images per launch of
the dominant kernel / that kernel's average launch time / 8 TB/s;
roofline.frac_end_to_end uses the whole step time; roofline.traffic is the
dominant kernel's HBM bytes per launch from the committed rocprofv3 PMC
passes (profiles/pmc_r06.json) and traffic_ratio = traffic / algorithmic.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_ACHIEVABLE_GBS = 6290.0  # MI355X_MICROARCH.md: 6.29 TB/s measured (float4 copy)
FP32_MFMA_PEAK_TF = 157.3    # dense fp32 MFMA (= vector) peak
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_r06.json")
CPU_CAL_FILE = os.path.join(ROOT, "profiles", "cpu_calibration_r02.json")


def launcher_command(argv, gpus, port=None):
    """The torchrun command that runs this bench on `gpus` ranks of one node
    (SURVEY §8(e)): a child process, never an exec of this one."""
    if port is None:
        so = socket.socket()
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
        so.close()
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def encode_bytes_per_image(h, w, t, ncb, s, images_per_row):
    """SURVEY §8(d) algorithmic bytes per image: fp32 RGB read + int64 codes,
    positions (2), channel, image id per token + key_pad_mask share."""
    return 12 * h * w + t * (8 * ncb + 32) + s / images_per_row


def kernel_models(h, w, p, maxp, ncb, s, images_per_row):
    """Algorithmic work per image of each kernel."""
    qh, qw = min(h // p, maxp), min(w // p, maxp)
    kh, kw = p * qh, p * qw
    t = 3 * qh * qw
    stage = t * (4 + 2 * ncb)            # score (f32) + LFQ codes (u16) per token, flat order
    inter = 12 * h * kw                   # row-pass output T: 3 channels x H x Kw fp32
    return {
        # name: (bound, per-image amount, unit) — DESIGN.md "Kernels"
        "rgb_to_ipt": ("hbm", 12 * h * w + 12 * h * w, "B"),
        "gemm_rows": ("mfma", 3 * 2.0 * kw * h * w, "flop"),
        "gemm_cols": ("mfma", 3 * 2.0 * kh * kw * h, "flop"),
        "fft_rows": ("hbm", 12 * h * w + inter, "B"),            # RGB in, T out
        "fft_cols": ("hbm", inter + stage, "B"),                  # T in, token staging out
        "tile_epilogue": ("hbm", 12 * kh * kw + stage, "B"),
        "sort_pack": ("hbm", stage + t * (8 * ncb + 32) + s / images_per_row, "B"),
        "pad_fill": ("hbm", s / images_per_row, "B"),
    }


def cpu_calibration():
    """profiles/cpu_calibration_r02.json (tools/calibrate_cpu_baseline.py): the
    port's speed against the reference itself, measured in the build container."""
    try:
        with open(CPU_CAL_FILE) as f:
            c = json.load(f)
        return {"port_over_reference": c["port_over_reference"], "threads": c["threads"],
                "reference_mpix_s": c["reference_mpix_s"], "port_mpix_s": c["port_mpix_s"],
                "where": "build container (tools/calibrate_cpu_baseline.py)"}
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline(size, seconds, pn_tables, threads):
    from oracle import ref_cpu
    torch.set_num_threads(threads)
    cfg = ref_cpu.FEConfig()
    lcfg = ref_cpu.LFQConfig()
    g = torch.Generator().manual_seed(0)
    n, t0 = 0, time.perf_counter()
    chunk = 8
    while True:
        imgs = [torch.rand(3, size, size, generator=g) for _ in range(chunk)]
        ref_cpu.encode(imgs, cfg, pn_tables, lcfg, batch_size=None, build_attn_mask=True)
        n += chunk
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    mpix = n * size * size / 1e6
    return {"value": round(mpix / el, 3), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"{n} images of {size}x{size} (torch.rand) through oracle/ref_cpu.encode: preprocess "
                      f"(FFT DCT, sort) + iter_batches (attn_mask built) + PatchNorm + LFQ, {el:.1f} s",
            "calibration": cpu_calibration()}


def cpu_config1(threads, reps=10, size=224):
    """BASELINE config 1: one 224x224 image through the reference's CPU round
    trip (FE:154-310: preprocess -> iter_batches(None) -> postprocess, DCT then
    IDCT) on the oracle port, median of ``reps`` runs."""
    from oracle import ref_cpu
    torch.set_num_threads(threads)
    cfg = ref_cpu.FEConfig()
    x = torch.rand(3, size, size, generator=torch.Generator().manual_seed(1))
    times, err = [], 0.0
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        item = ref_cpu.preprocess(x, cfg)
        (batch,) = list(ref_cpu.iter_batches(iter([{k: [v] for k, v in item.items()}]), cfg, None))
        (y,) = ref_cpu.postprocess(batch, cfg)
        times.append(time.perf_counter() - t0)
        err = float((y - x).abs().max())
    times = sorted(times[1:])   # the first run warms the allocator / thread pool
    med = times[len(times) // 2]
    return {"workload": f"config 1: one {size}x{size} image, preprocess -> iter_batches -> postprocess "
                        "(DCT -> IDCT round trip) on the CPU port", "median_ms": round(med * 1e3, 3),
            "reps": reps, "cores": threads, "kind": "port", "roundtrip_max_abs_err": err}


def cpu_config_legs(threads, tables, seed=3, min_s=2.0):
    """BASELINE.md §3's capped CPU subsets of configs 2-4 on the oracle port
    (the reference's op sequence: FFT DCT, per-image sort, greedy packing with
    attn_mask, PatchNorm, LFQ; decode through the reference's per-token revert
    loop, FE:639-643), each a few seconds of host time:
      config 2: 256 x 224^2 encode;
      config 3: 8 x 512^2 round trip (encode, then indices_to_codes ->
                inverse_norm -> postprocess), encode and decode timed apart;
      config 4: the first 32 images of the GPU leg's ragged sizes (seed 7).
    Each leg runs once untimed, then repeats until min_s of host time."""
    from oracle import ref_cpu
    torch.set_num_threads(threads)
    cfg, lcfg = ref_cpu.FEConfig(), ref_cpu.LFQConfig()
    g = torch.Generator().manual_seed(seed)
    out = {}

    def enc(imgs):
        return ref_cpu.encode(imgs, cfg, tables, lcfg, batch_size=None, build_attn_mask=True)

    def timed(fn, min_s):
        """fn repeated until min_s of host time (after one untimed run): mean seconds per run"""
        fn()
        n, t0 = 0, time.perf_counter()
        while True:
            fn()
            n += 1
            el = time.perf_counter() - t0
            if el >= min_s:
                return el / n, n

    imgs = [torch.rand(3, 224, 224, generator=g) for _ in range(256)]
    el, n = timed(lambda: enc(imgs), min_s)
    out["config2"] = {"workload": "256 x 224x224 encode", "value": round(256 * 224 * 224 / el / 1e6, 3),
                      "unit": "Mpix/s", "seconds_per_run": round(el, 4), "runs": n}
    imgs = [torch.rand(3, 512, 512, generator=g) for _ in range(8)]
    el_e, n_e = timed(lambda: enc(imgs), min_s)
    res = enc(imgs)

    def dec():
        n_out = 0
        for batch, idx in res:
            b = ref_cpu.Batch(None, batch.key_pad_mask, None, batch.batched_image_ids, batch.patch_channels,
                              batch.patch_positions, batch.patch_sizes, batch.original_sizes)
            y = ref_cpu.lfq_indices_to_codes(idx, lcfg)
            b.patches = ref_cpu.norm_inverse(tables, y, batch.patch_channels, batch.h_indices, batch.w_indices)
            n_out += len(ref_cpu.postprocess(b, cfg, per_token_loop=True))
        assert n_out == 8

    el_d, n_d = timed(dec, min_s)
    pix = 8 * 512 * 512
    out["config3"] = {"workload": "8 x 512x512 round trip (encode + decode through the per-token revert loop)",
                      "value": round(pix / (el_e + el_d) / 1e6, 3), "unit": "Mpix/s (round trip)",
                      "encode_mpix_s": round(pix / el_e / 1e6, 3), "decode_mpix_s": round(pix / el_d / 1e6, 3),
                      "seconds_per_run": round(el_e + el_d, 4), "runs": [n_e, n_d]}
    hw = np.random.default_rng(7).integers(14, 1025, size=(1024, 2))[:32]
    imgs = [torch.rand(3, int(h), int(w), generator=g) for h, w in hw]
    el, n = timed(lambda: enc(imgs), min_s)
    out["config4"] = {"workload": "32 ragged images, the GPU leg's first 32 sizes (H, W) ~ U{14..1024}^2 seed 7, "
                                  "encode", "value": round(int((hw[:, 0] * hw[:, 1]).sum()) / el / 1e6, 3),
                      "unit": "Mpix/s", "seconds_per_run": round(el, 4), "runs": n}
    return out


def stats_fit_leg(pkg, fe, dev, rank, world, dist, steps, n_img=8, size=512):
    """Config 5: one data-parallel PatchNorm fit step per
    iteration — each rank's batch statistics of its own shard, exchanged over
    RCCL (two all_gathers of the (3, 32, 32, 196) tables, distributed.py) and
    the running-update chain replayed locally.  At N = 1 a one-rank NCCL group
    runs the same code.  The shard's encode is outside the timed region."""
    from importlib import import_module
    import torch.distributed as tdist
    ops = import_module("dct_autoencoder_amd._ops")
    dd = import_module("dct_autoencoder_amd.distributed")
    own = False
    if not tdist.is_initialized():
        import socket
        so = socket.socket()
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
        so.close()
        tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
        own = True
    try:
        xs = ops.synth_images(n_img, size, size, seed=99, first_index=rank * n_img, device=dev)
        ((dp, _),) = fe.encode_batch(xs, None, None, return_raw=True)
        pn_t = pkg.PatchNorm(32, 32, 14, 3).to(dev).train()
        dd.train_step(pn_t, dp)                          # warm-up (plans, RCCL channels)
        torch.cuda.synchronize(dev)
        tdist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            dd.train_step(pn_t, dp)
        torch.cuda.synchronize(dev)
        tdist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        tdist.all_reduce(el, op=tdist.ReduceOp.MAX)
        # parity of the exchange: one fit step from empty tables
        # on every rank must equal, bit for bit, one process applying the
        # reference update (patchnorm.py:101-155, HIP stats kernels) to the
        # world's shards as consecutive batches in rank order
        pn_d = pkg.PatchNorm(32, 32, 14, 3).to(dev).train()
        dd.train_step(pn_d, dp)
        pn_s = pkg.PatchNorm(32, 32, 14, 3).to(dev).train()
        for r in range(world):
            xr = ops.synth_images(n_img, size, size, seed=99, first_index=r * n_img, device=dev)
            ((dpr, _),) = fe.encode_batch(xr, None, None, return_raw=True)
            pn_s(dpr)
        torch.cuda.synchronize(dev)
        same = all(torch.equal(getattr(pn_d, k).data, getattr(pn_s, k).data) for k in ("n", "median", "b"))
        flag = torch.tensor([1 if same else 0], dtype=torch.int32, device=dev)
        tdist.all_reduce(flag, op=tdist.ReduceOp.MIN)
        table_bytes = 3 * 32 * 32 * (14 * 14 + 1) * 4
        return {"workload": f"config 5 stats fit: PatchNorm running statistics of {n_img} x {size}x{size} images "
                            f"per rank, 2 all_gathers over {'RCCL' if tdist.get_backend() == 'nccl' else tdist.get_backend()} "
                            f"+ local replay of the update chain",
                "ranks": world, "ms_per_step": round(float(el.item()) / steps * 1e3, 4),
                "gathered_bytes_per_rank_per_step": 2 * table_bytes * world,
                "tables_bit_equal_to_sequential_fit": bool(flag.item()),
                "tokens_per_rank": int((~dp.key_pad_mask).sum().item())}
    finally:
        if own:
            tdist.destroy_process_group()


def config_legs(pkg, fe, pn, lfq, dev, rank, steps):
    """SURVEY §8(d) configs 2 and 4 on this GPU (informational; the metric is config 3's shape):
    config 2 = 256 x 224^2 encode (pre-planned BatchEncoder, inputs resident);
    config 4 = 1024 ragged images, (H, W) ~ U{14..1024}^2 (seed 7), encode_batch (host
    planning + packing included: the plan depends on the sizes)."""
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    fe_mod = import_module("dct_autoencoder_amd.feature_extraction")
    out = {}
    x2 = ops.synth_images(256, 224, 224, seed=1234, first_index=rank * 256, device=dev)
    enc2 = fe_mod.BatchEncoder(fe, 256, 224, 224, pn, lfq, device=dev)
    # a call is ~0.13 ms: 5 warm-up calls, then at least 200 timed back-to-back
    # calls (20 calls = 3 ms would time the clock ramp after the CPU legs)
    for _ in range(5):
        enc2(x2)
    torch.cuda.synchronize(dev)
    n2 = max(steps, 200)
    t0 = time.perf_counter()
    for _ in range(n2):
        enc2(x2)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / n2
    lib = import_module("dct_autoencoder_amd._lib")
    out["config2"] = {"workload": "256 x 224x224 encode", "ms_per_step": round(el * 1e3, 4), "calls": n2,
                      "value": round(256 * 224 * 224 / el / 1e6, 1), "unit": "Mpix/s",
                      "kernels": kernel_times(lib.context(dev), lambda: enc2(x2), 5)}
    g = np.random.default_rng(7)
    hw = g.integers(14, 1025, size=(1024, 2))
    imgs = [ops.synth_images(1, int(h), int(w), seed=7, first_index=rank * 1024 + i, device=dev)[0]
            for i, (h, w) in enumerate(hw)]
    fe.encode_batch(imgs, pn, lfq)
    torch.cuda.synchronize(dev)
    # back-to-back calls, steady state: each call's host planning / packing
    # (~2.7 ms for these 1024 sizes) overlaps the previous call's kernels.  A
    # warm-up call is enqueued first and the timed region runs on the stream
    # from its end (events) to the end of the n4 timed calls, so the first timed
    # call's planning overlaps the warm-up's kernels like every later one
    n4 = max(1, min(steps, 10))
    fe.encode_batch(imgs, pn, lfq)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(n4):
        fe.encode_batch(imgs, pn, lfq)
    e1.record()
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) / n4
    el = e0.elapsed_time(e1) / 1e3 / n4
    pix = int((hw[:, 0] * hw[:, 1]).sum())
    kern = kernel_times(lib.context(dev), lambda: fe.encode_batch(imgs, pn, lfq), 1)
    out["config4"] = {"workload": "1024 ragged images, (H, W) ~ U{14..1024}^2 seed 7, encode_batch incl. host packing",
                      "ms_per_step": round(el * 1e3, 3), "value": round(pix / el / 1e6, 1), "unit": "Mpix/s",
                      "host_wall_ms_per_call": round(wall * 1e3, 3),
                      "kernels": kern,
                      "device_ms": round(sum(v["total_ms"] for v in kern.values()), 3)}
    # conf/patch14-l.json's LFQ (16 codebooks of 2^13 over 196-element tokens: project_in
    # 196 -> 208, lfq.py:54-62) on the headline geometry: the fused encode stops at the
    # PatchNorm output and dctae_lfq_project_in (project_in + sign + pack) follows
    torch.manual_seed(0)
    lfq_p = type(lfq)(dim=196, codebook_size=2 ** 13, num_codebooks=16).to(dev).eval()
    x3 = ops.synth_images(1024, 512, 512, seed=1234, first_index=rank * 1024, device=dev)
    encp = fe_mod.BatchEncoder(fe, 1024, 512, 512, pn, lfq_p, device=dev)
    encp(x3)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        encp(x3)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / steps
    out["lfq_projections"] = {"workload": "1024 x 512x512 encode with conf/patch14-l.json's LFQ (16 x 2^13, "
                                          "project_in 196 -> 208 fused with sign / packing)",
                              "ms_per_step": round(el * 1e3, 4), "value": round(1024 * 512 * 512 / el / 1e6, 1),
                              "unit": "Mpix/s", "kernels": kernel_times(lib.context(dev), lambda: encp(x3), 5)}
    # and its decode: codes -> project_out (fused) -> inverse PatchNorm -> decode from tokens
    packed = encp(x3)
    decp = fe_mod.BatchDecoder(encp, pn, lfq_p)
    decp(packed)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        decp(packed)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / steps
    out["lfq_projections"]["decode"] = {
        "workload": "decode of those codes: codes -> project_out, the inverse PatchNorm inside the decode's column kernel (dctae_decode_normed), IDCT -> RGB",
        "ms_per_step": round(el * 1e3, 4), "value": round(1024 * 512 * 512 / el / 1e6, 1), "unit": "Mpix/s",
        "kernels": kernel_times(lib.context(dev), lambda: decp(packed), 5)}
    del x3, encp, decp, packed
    return out


def config5_leg(enc, dev, rank, world, dist, shard):
    """rank r encodes its shard of `shard` 512x512 images
    (global images [r*shard, (r+1)*shard)), regenerated from the counter RNG in
    1024-image chunks into one resident buffer; generation and encode timed
    separately with HIP events on the stream, max over ranks.  The stats-fit
    all-reduce step of config 5 is the `stats_fit` object."""
    import ctypes as C
    from importlib import import_module
    lib = import_module("dct_autoencoder_amd._lib")
    ctx = lib.context(dev)
    B, H = enc.B if hasattr(enc, "B") else 1024, 512
    n_chunks = max(1, shard // B)
    x = torch.empty((B, 3, H, H), dtype=torch.float32, device=dev)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(n_chunks)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(n_chunks):
        e = evs[i]
        e[0].record()
        rc = ctx.lib.dctae_synth_images(ctx.h, C.c_uint64(5), rank * shard + i * B, B, H, H,
                                        C.c_void_p(x.data_ptr()), lib.stream_ptr(dev))
        ctx.check(rc, "dctae_synth_images")
        e[1].record()
        enc(x)
        e[2].record()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    gen = sum(e[0].elapsed_time(e[1]) for e in evs) / 1e3
    encs = sum(e[1].elapsed_time(e[2]) for e in evs) / 1e3
    t = torch.tensor([encs, gen, wall], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    encs, gen, wall = (float(v) for v in t.tolist())
    imgs = n_chunks * B * world
    return {"workload": f"config 5: {world} rank(s) x {n_chunks * B} images of 512x512 (RNG-regenerated in "
                        f"{B}-image chunks), encode", "images": imgs,
            "encode_s": round(encs, 4), "generation_s": round(gen, 4), "wall_s": round(wall, 4),
            "value": round(imgs * H * H / encs / 1e6, 1), "unit": "Mpix/s (encode time, max over ranks)"}


def kernel_times(ctx, fn, n):
    """Per-kernel device times of n calls of fn (HIP events around each launch
    on its own stream, dctae_set_timing), outside any timed region."""
    import ctypes as C
    ctx.lib.dctae_timing_reset(ctx.h)
    ctx.lib.dctae_set_timing(ctx.h, 1)
    for _ in range(n):
        fn()
    ctx.lib.dctae_set_timing(ctx.h, 0)
    ctx.lib.dctae_timing_collect(ctx.h)
    out, i = {}, 0
    while True:
        name, ms, cnt = C.c_char_p(), C.c_double(), C.c_int64()
        if ctx.lib.dctae_timing_get(ctx.h, i, C.byref(name), C.byref(ms), C.byref(cnt)) != 0:
            break
        out[name.value.decode()] = {"total_ms": round(ms.value / n, 4), "launches": int(cnt.value) // n}
        i += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="images per GPU per step")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-decode", action="store_true", help="skip the config-3 decode timing")
    ap.add_argument("--no-stats", action="store_true", help="skip the config-5 PatchNorm fit (RCCL) timing")
    ap.add_argument("--model", action="store_true", help="also time the DCTAutoencoder transformer (SURVEY §8(f)4)")
    ap.add_argument("--no-model", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-configs", action="store_true", help="skip the config 2 / config 4 timings")
    ap.add_argument("--config5-shard", type=int, default=131072,
                    help="images per rank of the config-5 leg (0 = skip; SURVEY 8(d): 131,072 x 8 ranks)")
    ap.add_argument("--opt", action="append", default=[], help="library option key=value (dctae_set_option)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: torchrun as a child (nothing has touched the GPU yet)
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.call(launcher_command(sys.argv[1:], args.gpus), env=env))

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if os.environ.get("DCTAE_BENCH_SHARE_GPU"):   # rehearsal of N ranks on fewer GPUs (never in the driver's runs)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # RCCL refuses two ranks on one GPU: the shared-GPU rehearsal runs its
        # collectives on gloo (the driver's N-GPU runs always use nccl = RCCL)
        if os.environ.get("DCTAE_BENCH_SHARE_GPU") and torch.cuda.device_count() < world:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    import _pkgload
    pkg = _pkgload.load()
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    fe_mod = import_module("dct_autoencoder_amd.feature_extraction")

    P, MAXP, S = 14, 32, 3072
    fe = pkg.DCTAutoencoderFeatureExtractor(3, P, 0.0, MAXP, MAXP, S)
    tabs = np.load(os.path.join(ROOT, "tests", "golden", "patchnorm_ref.npz"))
    pn = pkg.PatchNorm(MAXP, MAXP, P, 3).to(dev)
    pn.median.data.copy_(torch.from_numpy(tabs["median"]))
    pn.b.data.copy_(torch.from_numpy(tabs["b"]))
    pn.n.data.copy_(torch.from_numpy(tabs["n"]))
    pn.frozen = True
    pn.eval()
    lfq = pkg.LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).to(dev).eval()

    B, H = args.batch, args.size
    x = ops.synth_images(B, H, H, seed=1234, first_index=rank * B, device=dev)
    for kv in args.opt:
        k, v = kv.split("=")
        ops.set_option(k, int(float(v)), dev)
    enc = fe_mod.BatchEncoder(fe, B, H, H, pn, lfq, device=dev)
    ctx = enc.ctx
    for _ in range(args.warmup):
        enc(x)
    torch.cuda.synchronize(dev)

    timing = not args.no_kernel_timing
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        enc(x)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    ops.check_device_errors(dev)
    if timing:
        # per-kernel device times (HIP events around each launch, on its stream) in a
        # separate pass: the event records stay out of the timed region above
        ctx.lib.dctae_timing_reset(ctx.h)
        ctx.lib.dctae_set_timing(ctx.h, 1)
        for _ in range(args.steps):
            enc(x)
        ctx.lib.dctae_set_timing(ctx.h, 0)
        ctx.lib.dctae_timing_collect(ctx.h)
    el_t = torch.tensor([el], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())

    imgs_per_row = max(1, S // enc.k)
    pix = args.steps * B * H * H * world
    mpix_s = pix / el / 1e6
    ms_step = el / args.steps * 1e3
    t_tok = enc.k
    per_img_bytes = encode_bytes_per_image(H, H, t_tok, 14, S, imgs_per_row)
    hbm_frac = (per_img_bytes * B * world * args.steps / el) / (HBM_PEAK_GBS * 1e9 * world)

    kernels, roof = {}, None
    if timing:
        import ctypes as C
        models = kernel_models(H, H, P, MAXP, 14, S, imgs_per_row)
        i = 0
        while True:
            name = C.c_char_p()
            ms = C.c_double()
            n = C.c_int64()
            if ctx.lib.dctae_timing_get(ctx.h, i, C.byref(name), C.byref(ms), C.byref(n)) != 0:
                break
            kernels[name.value.decode()] = {"total_ms": round(ms.value, 4), "launches": int(n.value),
                                            "avg_ms": round(ms.value / max(1, n.value), 5)}
            i += 1
        if kernels:
            # the dominant kernel of the encode; its roofline uses the metric's
            # algorithmic bytes for the images one launch covers
            dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
            imgs_per_launch = B * args.steps / kernels[dom]["launches"]
            per_launch = per_img_bytes * imgs_per_launch
            avg_s = kernels[dom]["avg_ms"] / 1e3
            ach = per_launch / avg_s / 1e9
            traffic, pmc_src, floor = None, None, None
            if os.path.exists(PMC_FILE):
                pmc = json.load(open(PMC_FILE))
                # design floor: the HBM bytes the shipped encode kernels move per
                # image (PMC, every kernel of this step) at the achievable 6.29 TB/s
                pk = pmc.get("kernels", {})
                moved = [pk[k]["hbm_bytes_per_image"] for k in kernels if pk.get(k, {}).get("hbm_bytes_per_image")]
                if moved:
                    fb = sum(moved)
                    floor_ms = fb * B / (HBM_ACHIEVABLE_GBS * 1e9) * 1e3
                    floor = {"ms_per_step": round(floor_ms, 4), "bytes_per_image": round(fb),
                             "kernels": [k for k in kernels if pk.get(k, {}).get("hbm_bytes_per_image")],
                             "frac_at_floor": round(per_img_bytes * B / (floor_ms / 1e3) / (HBM_PEAK_GBS * 1e9), 4),
                             "note": "PMC bytes of the encode kernels at 6.29 TB/s achievable: the end-to-end "
                                     "fraction this kernel design can reach (the intermediate T's HBM round trip "
                                     "included)"}
                ent = pk.get(dom)
                if ent and ent.get("hbm_bytes_per_image"):
                    # HBM bytes per launch from the committed rocprofv3 PMC passes (FETCH_SIZE x 2 + WRITE_SIZE,
                    # MI355X_MICROARCH.md gfx950 correction), scaled to this launch's image count
                    traffic = round(ent["hbm_bytes_per_image"] * imgs_per_launch)
                    pmc_src = os.path.relpath(PMC_FILE, ROOT)
            bound, amt, unit = kernel_models(H, H, P, MAXP, 14, S, imgs_per_row).get(dom, ("hbm", 0, "B"))
            roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "traffic_ratio": round(traffic / per_launch, 3) if traffic else None,
                    "traffic_source": pmc_src,
                    "per_launch": f"{per_launch:.6g} B = {per_img_bytes:g} B/img x {imgs_per_launch:g} images "
                                  f"(SURVEY 8(d) algorithmic bytes of the encode)",
                    "frac_end_to_end": round(hbm_frac, 4),
                    "kernel_own_bytes_per_launch": round(amt * imgs_per_launch),
                    "kernel_own_frac": round(amt * imgs_per_launch / avg_s / 1e9 / HBM_PEAK_GBS, 4)
                    if unit == "B" else None,
                    "design_floor_ms": floor["ms_per_step"] if floor else None,
                    "design_floor": floor}

    # config 3: decode of this step's codes back to RGB, timed the same way
    decode = None
    if not args.no_decode:
        try:
            dec = fe_mod.BatchDecoder(enc, pn, lfq)
            packed = enc(x)
            for _ in range(args.warmup):
                dec(packed)
            torch.cuda.synchronize(dev)
            if dist:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                dec(packed)
            torch.cuda.synchronize(dev)
            if dist:
                dist.barrier()
            el_d = time.perf_counter() - t0
            ops.check_device_errors(dev)
            dk = {}
            if timing:
                import ctypes as C
                ctx.lib.dctae_timing_reset(ctx.h)
                ctx.lib.dctae_set_timing(ctx.h, 1)
                for _ in range(args.steps):
                    dec(packed)
                ctx.lib.dctae_set_timing(ctx.h, 0)
                ctx.lib.dctae_timing_collect(ctx.h)
                i = 0
                while True:
                    name, ms, n = C.c_char_p(), C.c_double(), C.c_int64()
                    if ctx.lib.dctae_timing_get(ctx.h, i, C.byref(name), C.byref(ms), C.byref(n)) != 0:
                        break
                    dk[name.value.decode()] = {"avg_ms": round(ms.value / max(1, n.value), 5)}
                    i += 1
            el_t = torch.tensor([el_d], dtype=torch.float64, device=dev)
            if dist:
                dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
            el_d = float(el_t.item())
            dec_bytes = t_tok * (8 * 14 + 32) + S / imgs_per_row + 12 * H * H   # read codes + meta, write RGB
            decode = {"workload": f"config 3 decode: LFQ codes -> inverse PatchNorm -> IDCT -> RGB, {B} x {H}x{H}",
                      "value": round(args.steps * B * H * H * world / el_d / 1e6, 2), "unit": "Mpix/s",
                      "ms_per_step": round(el_d / args.steps * 1e3, 4),
                      "hbm_roofline_frac": round(dec_bytes * B * world * args.steps / el_d / (HBM_PEAK_GBS * 1e9 * world), 5),
                      "kernels": dk}
        except Exception as e:  # noqa: BLE001 — the encode line must still print
            decode = {"error": f"{type(e).__name__}: {e}"}

    stats = None
    if not args.no_stats:
        try:
            stats = stats_fit_leg(pkg, fe, dev, rank, world, dist, args.steps)
        except Exception as e:  # noqa: BLE001 — the encode line must still print
            stats = {"error": f"{type(e).__name__}: {e}"}

    configs = None
    if not args.no_configs:
        try:
            configs = config_legs(pkg, fe, pn, lfq, dev, rank, args.steps)
        except Exception as e:  # noqa: BLE001 — the encode line must still print
            configs = {"error": f"{type(e).__name__}: {e}"}

    if args.config5_shard > 0 and B == 1024 and H == 512:
        try:
            c5 = config5_leg(enc, dev, rank, world, dist, args.config5_shard)
        except Exception as e:  # noqa: BLE001 — the encode line must still print
            c5 = {"error": f"{type(e).__name__}: {e}"}
        configs = dict(configs or {})
        configs["config5"] = c5

    # the DCTAutoencoder transformer forward (patch14-l, 4 rows x 3072 tokens)
    model = None
    if args.model and not args.no_model:
        try:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import model_bench
            model = model_bench.run(rows=4, steps=3, warmup=1, dev=dev)
        except Exception as e:  # noqa: BLE001 — the encode line must still print
            model = {"error": f"{type(e).__name__}: {e}"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import ref_cpu
        threads = min(16, os.cpu_count() or 1)
        tables = ref_cpu.NormTables(torch.from_numpy(tabs["n"]), torch.from_numpy(tabs["median"]),
                                    torch.from_numpy(tabs["b"]))
        cpu = cpu_baseline(H, args.cpu_seconds, tables, threads)
        cpu["config1"] = cpu_config1(threads)
        cpu["configs"] = cpu_config_legs(threads, tables)
        # the GPU figure of each config beside its CPU sample (same units)
        oc = configs if isinstance(configs, dict) else {}
        gpu = {"config2": (oc.get("config2") or {}).get("value"), "config4": (oc.get("config4") or {}).get("value")}
        if decode and decode.get("ms_per_step"):
            gpu["config3"] = round(B * H * H / ((ms_step + decode["ms_per_step"]) / 1e3) / 1e6, 1)
        for k, v in gpu.items():
            if v and k in cpu["configs"]:
                cpu["configs"][k]["gpu_value"] = v
                cpu["configs"][k]["gpu_over_cpu"] = round(v / cpu["configs"][k]["value"], 1)

    if rank == 0:
        line = {
            "metric": "Mpix/s encode (DCT+PatchNorm+LFQ), patch14 512²; 1/2/4/8 GPU, %HBM roofline",
            "value": round(mpix_s, 2),
            "unit": "Mpix/s",
            "n_gpus": world,
            "ranks": {"world": world, "backend": (("nccl (RCCL)" if dist.get_backend() == "nccl" else dist.get_backend())
                                                  if world > 1 else None)},
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (counter-RNG uniform [0,1) RGB generated on device; reference-fitted PatchNorm tables)",
            "config": {"workload": f"fused encode of {H}x{H} RGB images, patch14, max_patch 32x32, S={S}, "
                                   f"LFQ 14 codebooks x 2^14, beta=0",
                       "images_per_gpu_per_step": B, "global_batch": B * world, "image_hw": [H, H],
                       "tokens_per_image": t_tok, "parallelism": f"dp{world} (image shards, no collective)"},
            "hbm_roofline_frac_encode": round(hbm_frac, 5),
            "encode_bytes_per_image": per_img_bytes,
            "roofline": roof,
            "cpu_baseline": cpu,
            "kernels": kernels,
            "decode": decode,
            "stats_fit": stats,
            "model": model,
            "other_configs": configs,
            "options": args.opt,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
