#!/usr/bin/env python3
"""Turn a GPU profiling run (gpurun_out/) into the committed evidence under
profiles/:  rocprof kernel stats (copied) and a PMC summary JSON with the
HBM traffic of every kernel (FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM,
WRITE_SIZE as is), per dispatch and per image.

    python tools/make_profiles.py <round-tag> <images-per-dispatch>
"""
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
imgs = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
gp = os.path.join(ROOT, "gpurun_out")
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)
# library timer names <- kernel symbols
NAMES = {"k_fft_rows2": "fft_rows", "k_fft_rows": "fft_rows", "k_fft_cols2": "fft_cols", "k_fft_cols": "fft_cols",
         "k_fft_cols4": "fft_cols", "k_fft_cols5": "fft_cols", "k_fft_cols6": "fft_cols", "k_fft_cols7": "fft_cols",
         "k_enc_pipe": "enc_pipe", "k_enc_pipe2": "enc_pipe", "k_sort_pack2": "sort_pack",
         "k_enc_fused": "enc_fused", "k_dec_map": "dec_map", "k_idct_cols512": "idct_cols", "k_idct_rows2": "idct_rows",
         "k_sort_pack": "sort_pack", "k_pad_fill": "pad_fill", "k_gemm_f32": "gemm", "k_rgb_to_ipt": "rgb_to_ipt",
         "k_tile_epilogue": "tile_epilogue", "k_synth": "synth", "k_norm_thresholds": "norm_thresholds"}
stats = os.path.join(gp, "prof", "run_kernel_stats.csv")
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(prof, f"rocprof_kernel_stats_{tag}.csv"))
raw = json.loads(subprocess.check_output([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"),
                                          os.path.join(gp, "pmc")]))
out = {"tag": tag, "images_per_dispatch": imgs,
       "note": "rocprofv3 --pmc, one counter group per run; hbm_read = FETCH_SIZE*1024*2 (gfx950 reports half of "
               "wide coalesced reads), hbm_write = WRITE_SIZE*1024; per-image = per dispatch / images in the dispatch",
       "kernels": {}}
for sym, d in raw.items():
    base = sym.replace("void ", "").split("<")[0].split("::")[-1]
    name = NAMES.get(base, base)
    big = d.get("dispatches", 1) and d.get("SQ_WAVES", 0) > 1000
    ent = {"symbol": sym, **{k: v for k, v in d.items()}}
    if "hbm_read_bytes_corrected" in d and "hbm_write_bytes" in d:
        ent["hbm_bytes_per_dispatch"] = d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"]
        if big and name in ("fft_rows", "fft_cols", "sort_pack", "pad_fill", "gemm", "tile_epilogue", "rgb_to_ipt",
                            "enc_fused", "dec_map", "idct_cols", "idct_rows"):
            ent["images_per_dispatch"] = imgs
            ent["hbm_bytes_per_image"] = ent["hbm_bytes_per_dispatch"] / imgs
    out["kernels"][name if name not in out["kernels"] else sym] = ent
json.dump(out, open(os.path.join(prof, f"pmc_{tag}.json"), "w"), indent=1)
print(json.dumps({k: {kk: v.get(kk) for kk in ("hbm_bytes_per_image", "SQ_WAVES")} for k, v in out["kernels"].items()},
                 indent=1))
