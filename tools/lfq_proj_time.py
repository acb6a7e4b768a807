"""Time the fused LFQ projection kernels (dctae_lfq_project_in / _out) against
the unfused torch path (hipBLASLt nn.Linear + the HIP sign / codes kernels) on
the conf/patch14-l.json shape: 196 -> 16 x 13, tokens of 1024 512^2 images
(3,145,728 tokens).  Prints one JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
from dct_autoencoder_amd import _ops  # noqa: E402

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024 * 3072
torch.manual_seed(0)
m = pkg.LFQ(dim=196, codebook_size=2 ** 13, num_codebooks=16).to(dev).eval()
x = torch.randn(n, 196, device=dev)
cfg = m.cfg()
wi, bi = m._proj_w(m.project_in, dev)
wo, bo = m._proj_w(m.project_out, dev)


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


idx = _ops.lfq_project_in(x, wi, bi, cfg)
res = {
    "tokens": n,
    "fused_project_in_ms": t(lambda: _ops.lfq_project_in(x, wi, bi, cfg)),
    "torch_linear_plus_sign_ms": t(lambda: _ops.lfq_forward(torch.nn.functional.linear(x, wi, bi), cfg,
                                                              want_quantized=False)),
    "fused_project_out_ms": t(lambda: _ops.lfq_project_out(idx, wo, bo, cfg)),
    "torch_codes_plus_linear_ms": t(lambda: torch.nn.functional.linear(_ops.lfq_codes(idx, cfg), wo, bo)),
}
fl = 2.0 * n * 196 * 208
res["fused_project_in_tflops"] = fl / res["fused_project_in_ms"] / 1e9
res["fused_project_out_tflops"] = fl / res["fused_project_out_ms"] / 1e9
same = (torch.equal(_ops.lfq_project_in(x, wi, bi, cfg), idx))
res["deterministic"] = bool(same)
print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}))
