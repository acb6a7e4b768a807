"""MI355X-native drop-in for the feature-extraction hot path of
theAdamColton/dct-autoencoder (RGB -> IPT -> DCT -> spectral patches ->
PatchNorm -> LFQ and back), running on hand-written gfx950 HIP kernels
(libdctae.so, C ABI in include/dctae.h).

Import name: ``dct_autoencoder_amd`` (the directory is dct-autoencoder_amd/;
see _pkgload.py at the repository root)."""
from ._lib import DCTAEError, DCTAEUnavailable, load_library  # noqa: F401
from .dct_patches import DCTPatches, build_attn_mask, from_dict, to_dict  # noqa: F401
from .feature_extraction import DCTAutoencoderFeatureExtractor, GroupPatchesState  # noqa: F401
from .lfq import LFQ  # noqa: F401
from .model import CLIPEncoderConfig, DCTAutoencoder, DCTAutoencoderConfig  # noqa: F401
from .patchnorm import PatchNorm  # noqa: F401
from .vector_quantize import VectorQuantize  # noqa: F401
from . import packing  # noqa: F401
from . import shards  # noqa: F401

__all__ = ["DCTAutoencoderFeatureExtractor", "DCTPatches", "PatchNorm", "LFQ", "VectorQuantize", "to_dict", "from_dict",
           "DCTAutoencoder", "DCTAutoencoderConfig", "CLIPEncoderConfig",
           "GroupPatchesState", "build_attn_mask", "load_library", "DCTAEError", "DCTAEUnavailable"]
