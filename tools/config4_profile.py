import sys, time, json, ctypes as C
sys.path.insert(0, "."); import numpy as np, torch, _pkgload
pkg = _pkgload.load()
from importlib import import_module
ops = import_module("dct_autoencoder_amd._ops"); L = import_module("dct_autoencoder_amd._lib")
dev = torch.device("cuda", 0)
tabs = np.load("tests/golden/patchnorm_ref.npz")
pn = pkg.PatchNorm(32, 32, 14, 3).to(dev); pn.median.data.copy_(torch.from_numpy(tabs["median"])); pn.b.data.copy_(torch.from_numpy(tabs["b"])); pn.frozen = True; pn.eval()
lfq = pkg.LFQ(dim=196, codebook_size=2**14, num_codebooks=14).to(dev).eval()
fe = pkg.DCTAutoencoderFeatureExtractor(3, 14, 0.0, 32, 32, 3072)
g = np.random.default_rng(7); hw = g.integers(14, 1025, size=(1024, 2))
imgs = [ops.synth_images(1, int(h), int(w), seed=7, first_index=i, device=dev)[0] for i, (h, w) in enumerate(hw)]
fe.encode_batch(imgs, pn, lfq); torch.cuda.synchronize()
ctx = L.context(dev); ctx.lib.dctae_timing_reset(ctx.h); ctx.lib.dctae_set_timing(ctx.h, 1)
t0 = time.perf_counter(); fe.encode_batch(imgs, pn, lfq); t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
ctx.lib.dctae_set_timing(ctx.h, 0); ctx.lib.dctae_timing_collect(ctx.h)
i = 0; k = {}
while True:
    name, ms, n = C.c_char_p(), C.c_double(), C.c_int64()
    if ctx.lib.dctae_timing_get(ctx.h, i, C.byref(name), C.byref(ms), C.byref(n)) != 0: break
    k[name.value.decode()] = (round(ms.value, 3), n.value); i += 1
print("host enqueue ms", round((t1 - t0) * 1e3, 2), "total ms", round((t2 - t0) * 1e3, 2))
print(json.dumps(k))
from math import gcd
def smooth(n):
    for p in (2, 3, 5, 7):
        while n % p == 0: n //= p
    return n == 1
print("7-smooth even H and W:", sum(1 for h, w in hw if h % 2 == 0 and w % 2 == 0 and smooth(h) and smooth(w)))
