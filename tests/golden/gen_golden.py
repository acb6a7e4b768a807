"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
implementation (theAdamColton/dct-autoencoder, read-only at /root/reference)
in the build container.  See refload.py for how it is loaded.

    python tests/golden/gen_golden.py

Inputs are regenerated from the counter-based RNG in oracle/rng.py (so only
outputs are stored), except the real-image crops, which are stored as uint8.
Outputs are data only (arrays / JSON); no reference source is stored.
"""
import hashlib
import json
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import refload  # noqa: E402
from oracle import rng as orng  # noqa: E402

P, MAXP, S = 14, 32, 3072
CAL_SIZES = [(448, 448)] * 8 + [(300, 448), (448, 200), (150, 150), (460, 470)]
CASES = {
    "sq224": dict(seed=1234, first=0, sizes=[(224, 224), (224, 224)]),
    "ragged": dict(seed=7, first=0, sizes=[(30, 700), (100, 100), (300, 500), (14, 14), (15, 29), (57, 43)]),
    "sq512": dict(seed=1234, first=100, sizes=[(512, 512)]),
}
REAL = [("books.jpeg", 0, 0, 252, 308), ("dune.jpg", 40, 60, 224, 266)]
BETA_SIZES = [(224, 224), (100, 300), (512, 140), (64, 64), (300, 300), (28, 28)]
PACK_SIZES = [(224, 224), (100, 300), (512, 140), (64, 64), (300, 300), (28, 28), (150, 420), (90, 90)]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    ref = refload.load()
    FE = ref.fe.DCTAutoencoderFeatureExtractor
    PatchNorm = ref.patchnorm.PatchNorm
    LFQ = ref.lfq.LFQ
    util = ref.util
    torch.set_num_threads(8)

    def dict_collate(rows):
        return {k: [r[k] for r in rows] for k in rows[0]}

    # ---------------- colour matrices -------------------------------------
    np.savez(os.path.join(HERE, "colors.npz"),
             rgb2lms=util.Trgb2lms.numpy(), lms2rgb=util.Tlms2rgb.numpy(),
             lms2ipt=util.Mipt.numpy(), ipt2lms=util.Mipt.inverse().numpy())

    # ---------------- PatchNorm fitted by the reference training path -----
    proc = FE(3, P, 0.0, MAXP, MAXP, S)
    cal = orng.synth_images(99, CAL_SIZES)
    items = [proc.preprocess(torch.from_numpy(x)) for x in cal]
    loader = [dict_collate(items[i:i + 4]) for i in range(0, len(items), 4)]
    pn = PatchNorm(MAXP, MAXP, P, 3)
    pn.train()
    steps = 0
    for batch in proc.iter_batches(iter(loader), 4):
        pn(batch)
        steps += 1
    pn.frozen = True
    pn.eval()
    np.savez_compressed(os.path.join(HERE, "patchnorm_ref.npz"),
                        n=pn.n.data.numpy(), median=pn.median.data.numpy(), b=pn.b.data.numpy(),
                        steps=np.array(steps))
    meta = {"patchnorm": {"steps": steps, "cal_seed": 99, "cal_sizes": CAL_SIZES,
                          "sha_median": sha(pn.median.data.numpy()), "sha_b": sha(pn.b.data.numpy()),
                          "sha_n": sha(pn.n.data.numpy())}}

    lfq = LFQ(dim=196, codebook_size=2 ** 14, num_codebooks=14).eval()

    # ---------------- encode / decode cases --------------------------------
    def run_case(name, images, store_patches=True, store_rgb=True, sample_tokens=None):
        out = {}
        items = [proc.preprocess(torch.from_numpy(x)) for x in images]
        for i, it in enumerate(items):
            pt = it["patches"].numpy()
            if store_patches:
                out[f"img{i}_patches"] = pt
            elif sample_tokens:
                out[f"img{i}_patches_head"] = pt[:sample_tokens]
            out[f"img{i}_patches_sha"] = np.frombuffer(bytes.fromhex(sha(pt)), dtype=np.uint8)
            out[f"img{i}_positions"] = it["positions"].numpy().astype(np.int16)
            out[f"img{i}_channels"] = it["channels"].numpy().astype(np.int8)
            out[f"img{i}_original_size"] = np.array(it["original_sizes"])
            out[f"img{i}_patch_size"] = np.array(it["patch_sizes"])
        batches = list(proc.iter_batches(iter([dict_collate(items)]), None))
        assert len(batches) == 1
        batch = batches[0]
        out["key_pad_mask"] = batch.key_pad_mask.numpy()
        out["batched_image_ids"] = batch.batched_image_ids.numpy().astype(np.int16)
        out["patch_positions"] = batch.patch_positions.numpy().astype(np.int16)
        out["patch_channels"] = batch.patch_channels.numpy().astype(np.int8)
        raw = batch.shallow_copy()
        # round trip without quantisation (DCT -> IDCT)
        rt = proc.postprocess(raw)
        # encode: PatchNorm (eval) -> LFQ (eval)
        nb = batch.shallow_copy()
        nb.patches = pn(nb)
        q, idx, _, _ = lfq(nb.patches, mask=~nb.key_pad_mask)
        out["indices"] = idx.numpy().astype(np.int16)
        # decode from the reference's own codes
        db = nb.shallow_copy()
        db.patches = lfq.indices_to_codes(idx)
        assert torch.equal(db.patches, q)
        db.patches = pn.inverse_norm(db)
        dec = proc.postprocess(db)
        for i, (a, b) in enumerate(zip(rt, dec)):
            if store_rgb and a.shape[1] * a.shape[2] <= 60000 and (i == 0 or a.shape[1] * a.shape[2] <= 12000):
                out[f"img{i}_roundtrip_rgb"] = a.numpy()
                out[f"img{i}_decoded_rgb"] = b.numpy()
            out[f"img{i}_roundtrip_sha"] = np.frombuffer(bytes.fromhex(sha(a.numpy())), dtype=np.uint8)
        np.savez_compressed(os.path.join(HERE, f"case_{name}.npz"), **out)
        # codes as the reference's JSON code dump (dct_patches.to_dict)
        if name == "ragged":
            objs = ref.dct_patches.to_dict(nb, idx)
            with open(os.path.join(HERE, "ragged_to_dict.json"), "w") as f:
                json.dump(objs, f)
        return len(items)

    for name, c in CASES.items():
        imgs = orng.synth_images(c["seed"], c["sizes"], c["first"])
        big = name == "sq512"
        run_case(name, imgs, store_patches=not big, store_rgb=not big, sample_tokens=128)
        meta[name] = c

    from PIL import Image
    real = []
    for fn, y0, x0, hh, ww in REAL:
        im = np.asarray(Image.open(os.path.join(refload.REF, "images", fn)).convert("RGB"))
        real.append(np.ascontiguousarray(im[y0:y0 + hh, x0:x0 + ww].transpose(2, 0, 1)))
    np.savez_compressed(os.path.join(HERE, "real_inputs.npz"), **{f"img{i}": r for i, r in enumerate(real)})
    run_case("real", [r.astype(np.float32) / 255.0 for r in real], store_rgb=False)
    meta["real"] = {"crops": REAL}

    # ---------------- beta > 0 : k drawn from python random ----------------
    proc_b = FE(3, P, 0.02, MAXP, MAXP, 1024)
    random.seed(42)
    imgs = orng.synth_images(5, BETA_SIZES)
    out = {}
    for i, x in enumerate(imgs):
        it = proc_b.preprocess(torch.from_numpy(x))
        out[f"img{i}_positions"] = it["positions"].numpy().astype(np.int16)
        out[f"img{i}_channels"] = it["channels"].numpy().astype(np.int8)
        out[f"img{i}_k"] = np.array(it["patches"].shape[0])
    np.savez_compressed(os.path.join(HERE, "case_beta.npz"), **out)
    meta["beta"] = {"seed_python_random": 42, "beta": 0.02, "max_seq_len": 1024, "img_seed": 5,
                    "sizes": BETA_SIZES}

    # ---------------- packing / iter_batches quirks ------------------------
    proc_p = FE(3, P, 0.0, MAXP, MAXP, 1024)
    imgs = orng.synth_images(11, PACK_SIZES)
    items = [proc_p.preprocess(torch.from_numpy(x)) for x in imgs]
    out = {}
    scenarios = {
        "one_item_none": ([items], None),
        "two_items_none": ([items[:4], items[4:]], None),
        "items_b2": ([items[:3], items[3:6], items[6:]], 2),
        "items_b1": ([items[:2], items[2:5], items[5:]], 1),
    }
    for sname, (chunks, bs) in scenarios.items():
        loader = [dict_collate(ch) | {"tag": [f"t{j}" for j in range(len(ch))]} for ch in chunks]
        for bi, batch in enumerate(proc_p.iter_batches(iter(loader), bs)):
            pre = f"{sname}_b{bi}_"
            out[pre + "key_pad_mask"] = batch.key_pad_mask.numpy()
            out[pre + "ids"] = batch.batched_image_ids.numpy().astype(np.int16)
            out[pre + "positions"] = batch.patch_positions.numpy().astype(np.int16)
            out[pre + "channels"] = batch.patch_channels.numpy().astype(np.int8)
            out[pre + "attn_sha"] = np.frombuffer(bytes.fromhex(sha(batch.attn_mask.numpy())), dtype=np.uint8)
            out[pre + "original_sizes"] = np.array(batch.original_sizes).reshape(-1, 2)
            out[pre + "patch_sizes"] = np.array(batch.patch_sizes).reshape(-1, 2)
            out[pre + "data_tag"] = np.array(batch._data.get("tag", []))
        out[sname + "_nbatches"] = np.array(bi + 1 if chunks else 0)
    np.savez_compressed(os.path.join(HERE, "case_packing.npz"), **out)
    meta["packing"] = {"img_seed": 11, "sizes": PACK_SIZES, "max_seq_len": 1024}

    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
