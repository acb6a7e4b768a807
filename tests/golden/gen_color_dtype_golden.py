"""Golden vectors for FE._transform_image_in on fp16 / bf16 inputs: the
reference runs util.rgb_to_ipt in the INPUT dtype before ``x.float()``
(feature_extraction_dct_autoencoder.py:135-141), then dct2 in fp32 and casts
back.  Produced by running the REFERENCE in the build container (refload.py).

    python tests/golden/gen_color_dtype_golden.py  ->  tests/golden/color_dtype_ref.npz

Stored as fp32 arrays holding the dtype's values exactly: the inputs, the
reference's rgb_to_ipt output (in the dtype) and its _transform_image_in
output (in the dtype).  Data only; no reference source is stored.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import refload  # noqa: E402
from oracle import rng  # noqa: E402

SIZES = [(40, 56), (33, 70)]


def main():
    ref = refload.load()
    fe = ref.fe.DCTAutoencoderFeatureExtractor(channels=3, patch_size=14, sample_patches_beta=0.0,
                                               max_patch_h=32, max_patch_w=32, max_seq_len=3072)
    out = {}
    for tag, dt in (("f16", torch.float16), ("bf16", torch.bfloat16)):
        for i, x in enumerate(rng.synth_images(4321, SIZES)):
            xt = torch.from_numpy(x).to(dt)
            out[f"{tag}_{i}_x"] = xt.float().numpy()
            out[f"{tag}_{i}_ipt"] = ref.util.rgb_to_ipt(xt.clone()).float().numpy()
            y = fe._transform_image_in(xt.clone())
            assert y.dtype == dt
            out[f"{tag}_{i}_spec"] = y.float().numpy()
    path = os.path.join(HERE, "color_dtype_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
