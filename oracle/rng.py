"""Counter-based synthetic-image RNG (numpy) — TEST INFRASTRUCTURE ONLY.

The same hash is implemented on the GPU by ``dctae_synth_images`` in
``dct-autoencoder_amd/csrc/dctae.hip`` so the GPU box can regenerate bit-identical
inputs without shipping pixel arrays.  SURVEY §8(c) "counter-based RNG
(documented hash -> float = (u>>8)*2^-24)".

    key(seed, img)   = splitmix64(splitmix64(seed) ^ img)
    u(seed, img, e)  = splitmix64(key + e)            (e = flat index in (3,H,W))
    value            = (u >> 40) * 2**-24             (uniform on [0, 1), 24 bits)
"""
import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def image_key(seed: int, img: int) -> np.uint64:
    return splitmix64(splitmix64(np.uint64(seed)) ^ np.uint64(img))


def synth_image(seed: int, img: int, h: int, w: int, c: int = 3) -> np.ndarray:
    """(c, h, w) float32 in [0, 1)."""
    k = image_key(seed, img)
    e = np.arange(c * h * w, dtype=np.uint64)
    with np.errstate(over="ignore"):
        u = splitmix64(k + e)
    v = (u >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    return v.reshape(c, h, w)


def synth_images(seed: int, sizes, first_index: int = 0, c: int = 3):
    return [synth_image(seed, first_index + i, h, w, c) for i, (h, w) in enumerate(sizes)]


def ragged_sizes(seed: int, n: int, lo: int = 14, hi: int = 1024):
    """Config 4 sizes: (H, W) ~ U{lo..hi}^2 from the same hash (BASELINE config 4, seed 7)."""
    k = splitmix64(np.uint64(seed) ^ np.uint64(0xA5A5A5A5))
    with np.errstate(over="ignore"):
        u = splitmix64(k + np.arange(2 * n, dtype=np.uint64))
    span = np.uint64(hi - lo + 1)
    v = (u % span).astype(np.int64) + lo
    return [(int(v[2 * i]), int(v[2 * i + 1])) for i in range(n)]
