"""IPT colour matrices, built in fp32 exactly as the reference builds them
(reference dct_autoencoder/util.py:21-43, 91).  They are handed to the HIP
kernels as constants; the per-pixel transform itself runs on the GPU."""
import functools

import torch

# Published colour-science constants (sRGB->XYZ D65, Hunt-Pointer-Estevez
# XYZ->LMS, Ebner-Fairchild LMS'->IPT).
SRGB_TO_XYZ = ((0.4124564, 0.3575761, 0.1804375),
               (0.2126729, 0.7151522, 0.0721750),
               (0.0193339, 0.1191920, 0.9503041))
XYZ_TO_LMS = ((0.4002, 0.7076, -0.0807), (-0.2280, 1.1500, 0.0612), (0.0, 0.0, 0.9184))
LMS_TO_IPT = ((0.4, 0.4, 0.2), (4.455, -4.851, 0.3960), (0.8056, 0.3572, -1.1628))
IPT_GAMMA = 0.43


@functools.lru_cache(maxsize=1)
def matrices():
    srgb = torch.tensor(SRGB_TO_XYZ, dtype=torch.float32)
    hpe = torch.tensor(XYZ_TO_LMS, dtype=torch.float32)
    ipt = torch.tensor(LMS_TO_IPT, dtype=torch.float32)
    rgb2lms = hpe @ srgb
    return {"rgb2lms": rgb2lms, "lms2rgb": rgb2lms.inverse(), "lms2ipt": ipt, "ipt2lms": ipt.inverse()}
