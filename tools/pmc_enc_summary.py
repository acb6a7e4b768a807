"""Per-kernel summary of tools/gpu_pmc_enc.sh passes: counter values per
dispatch (averaged over the dispatches of a kernel).  FETCH_SIZE / WRITE_SIZE
are KiB; FETCH_SIZE is doubled per MI355X_MICROARCH.md §HBM (gfx950 reports
half of wide coalesced streaming reads).  With --profile OUT it also writes
the bench-readable profile (profiles/pmc_rNN.json): per library timer name
the HBM bytes per dispatch and per image.

    python tools/pmc_enc_summary.py <pmc dir> [--profile OUT --images N --tag rNN]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

# library timer names (dctae_set_timing) <- kernel symbols
NAMES = {"k_rows512": "fft_rows", "k_rows512pk": "fft_rows", "k_fft_rows2": "fft_rows", "k_fft_rows": "fft_rows", "k_fft_cols7": "fft_cols", "k_cols512b": "fft_cols",
         "k_fft_cols4": "fft_cols", "k_rows224p": "fft_rows", "k_cols224": "fft_cols", "k_fft_cols": "fft_cols", "k_sort_pack2": "sort_pack", "k_sort_pack": "sort_pack",
         "k_pad_fill": "pad_fill", "k_dec_map": "dec_map", "k_idct_cols512": "idct_cols", "k_idct_rows2": "idct_rows", "k_idct_rows512": "idct_rows",
         "k_gemm_f32": "gemm", "k_rgb_to_ipt": "rgb_to_ipt", "k_tile_epilogue_p": "tile_epilogue",
         "k_tile_epilogue": "tile_epilogue", "k_gemm_x3": "gemm", "k_idct_cols512b": "idct_cols", "k_gemm_h2": "gemm",
         "k_lfq_ws": "lfq_ws", "k_lfq_proj_h2": "lfq_proj_h2", "k_lfq_proj": "lfq_proj"}

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--profile")
ap.add_argument("--images", type=int, default=1024)
ap.add_argument("--tag", default="r02")
args = ap.parse_args()
acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(set))
for f in glob.glob(os.path.join(args.dir, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        short = name.split("(")[0].replace("void ", "").replace("dctae::", "")
        key = r["Counter_Name"]
        acc[short][key] += float(r["Counter_Value"])
        cnt[short][key].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
res = {}
for k, d in acc.items():
    res[k] = {}
    for c, v in d.items():
        v = v / max(1, len(cnt[k][c]))
        if c == "FETCH_SIZE":
            v *= 2.0
        res[k][c] = round(v, 1)
json.dump(res, open(os.path.join(args.dir, "summary.json"), "w"), indent=1)
for k, d in res.items():
    if any(s in k for s in ("rows", "cols", "sort", "pad", "dec_map", "gemm", "rgb", "epilogue")):
        print(k[:48], json.dumps(d))
if args.profile:
    out = {"tag": args.tag, "images_per_dispatch": args.images,
           "note": "rocprofv3 --pmc, one counter group per run, encode of 1024 x 512^2 (bench.py encode leg); "
                   "hbm_read = FETCH_SIZE * 1024 * 2 (gfx950 reports half of wide coalesced reads), hbm_write = "
                   "WRITE_SIZE * 1024; per image = per dispatch / images per dispatch",
           "kernels": {}}
    for sym, d in res.items():
        base = sym.split("<")[0]
        name = NAMES.get(base, base)
        ent = {"symbol": sym, **d}
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            ent["hbm_read_bytes"] = d["FETCH_SIZE"] * 1024
            ent["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
            ent["hbm_bytes_per_dispatch"] = ent["hbm_read_bytes"] + ent["hbm_write_bytes"]
            if d.get("SQ_WAVES", 0) > 1000:
                ent["images_per_dispatch"] = args.images
                ent["hbm_bytes_per_image"] = ent["hbm_bytes_per_dispatch"] / args.images
        if "SQ_LDS_BANK_CONFLICT" in d and d.get("SQ_LDS_IDX_ACTIVE"):
            ent["lds_bank_conflict_share"] = round(d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"], 4)
        out["kernels"][name if name not in out["kernels"] else sym] = ent
    json.dump(out, open(args.profile, "w"), indent=1)
