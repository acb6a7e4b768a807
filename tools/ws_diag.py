"""Diagnose k_lfq_ws mode 0 against k_lfq_proj_h2 on the same bounded input
(dctae_lfq_project_in_bounded with option lfq_ws 1 / 0): mismatch counts by
token position within a 64-token tile, by codebook and by token."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import _pkgload
    pkg = _pkgload.load()
    from importlib import import_module
    ops = import_module("dct_autoencoder_amd._ops")
    dev = torch.device("cuda", 0)
    torch.manual_seed(5)
    m = pkg.LFQ(dim=196, codebook_size=2 ** 13, num_codebooks=16).to(dev).eval()
    w, b = m._proj_w(m.project_in, dev)
    cfg = m.cfg(m.project_in.weight.dtype)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3 * 3072
    x = (torch.rand(n, 196, device=dev) * 12 - 6)
    out = {}
    for v in (0, 1):
        ops.set_option("lfq_ws", v, dev)
        out[v] = ops.lfq_project_in(x, w, b, cfg, 6.0).cpu()
    ops.set_option("lfq_ws", 1, dev)
    ref = torch.nn.functional.linear(x.cpu(), w.cpu(), b.cpu())
    bits_ref = (ref > 0).view(n, 16, 13)
    mask = 2 ** torch.arange(12, -1, -1)
    idx_ref = (bits_ref.long() * mask).sum(-1)
    for v in (0, 1):
        d = out[v] != idx_ref
        print(f"lfq_ws={v}: codes != fp32 linear: {int(d.sum())} / {d.numel()}")
    d = out[1] != out[0]
    print("ws vs h2 mismatches:", int(d.sum()))
    if d.any():
        tok = torch.nonzero(d.any(-1)).flatten()
        print("tokens:", tok[:40].tolist())
        print("by token % 64:", torch.bincount(tok % 64, minlength=64).tolist())
        print("by codebook:", d.sum(0).tolist())
        t = int(tok[0])
        print("token", t, "ws", out[1][t].tolist(), "h2", out[0][t].tolist(), "ref", idx_ref[t].tolist())


if __name__ == "__main__":
    main()
