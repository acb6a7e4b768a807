"""Load the reference's own Python (read-only, from /root/reference) for golden
vector generation.  BUILD-CONTAINER ONLY: the GPU box has no /root/reference,
and nothing under tests/ that runs there imports this module.

Recipe from SURVEY.md §8(c):
  1. a synthetic package object ``dct_autoencoder`` whose __path__ points at the
     reference sources (skips its __init__, which pulls in the CLIP model);
  2. ``util.py`` is executed with one syntax backport (reference util.py:344
     uses the Python-3.11 form ``y[..., *[...]]``; this container has 3.10);
  3. a ``torchvision`` stub (only used by off-path image-grid helpers);
  4. a ``torch_dct`` module restating torch_dct==0.1.6 (reference
     requirements.txt:13; not installed here, no network).  The restatement is
     ``oracle.ref_cpu.dct_1d``/``idct_1d``; it is pinned independently against
     ``scipy.fft.dctn`` in float64 (tests/test_oracle.py).
Nothing from the reference is copied into this repository.
"""
import importlib
import os
import sys
import types

REF = "/root/reference"


def available() -> bool:
    return os.path.isdir(os.path.join(REF, "dct_autoencoder"))


def load():
    if "dct_autoencoder.feature_extraction_dct_autoencoder" in sys.modules:
        return _handles()
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(os.path.dirname(here))
    if root not in sys.path:
        sys.path.insert(0, root)
    from oracle import ref_cpu

    # let transformers run its optional-dependency probes before the stub exists
    import transformers.feature_extraction_utils  # noqa: F401
    import transformers.configuration_utils  # noqa: F401
    import importlib.machinery

    tv = types.ModuleType("torchvision")
    tv.__spec__ = importlib.machinery.ModuleSpec("torchvision", None)
    tv.transforms = types.ModuleType("torchvision.transforms")
    tv.utils = types.ModuleType("torchvision.utils")
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.transforms", tv.transforms)
    sys.modules.setdefault("torchvision.utils", tv.utils)

    tdct = types.ModuleType("torch_dct")
    tdct.dct = lambda x, norm=None: ref_cpu.dct_1d(x)
    tdct.idct = lambda x, norm=None: ref_cpu.idct_1d(x)

    def dct_2d(x, norm=None):
        assert norm == "ortho"
        return ref_cpu.dct2(x)

    def idct_2d(x, norm=None):
        assert norm == "ortho"
        return ref_cpu.idct2(x)

    tdct.dct_2d = dct_2d
    tdct.idct_2d = idct_2d
    sys.modules["torch_dct"] = tdct

    pkg = types.ModuleType("dct_autoencoder")
    pkg.__path__ = [os.path.join(REF, "dct_autoencoder")]
    sys.modules["dct_autoencoder"] = pkg

    util_path = os.path.join(REF, "dct_autoencoder", "util.py")
    with open(util_path) as f:
        src = f.read()
    src = src.replace("y[..., *[None for _ in range(ndim_to_expand)]]",
                      "y[(Ellipsis, *[None for _ in range(ndim_to_expand)])]")
    util = types.ModuleType("dct_autoencoder.util")
    util.__file__ = util_path
    util.__package__ = "dct_autoencoder"
    exec(compile(src, util_path, "exec"), util.__dict__)
    sys.modules["dct_autoencoder.util"] = util
    pkg.util = util
    return _handles()


def _handles():
    fe = importlib.import_module("dct_autoencoder.feature_extraction_dct_autoencoder")
    pn = importlib.import_module("dct_autoencoder.patchnorm")
    lfq = importlib.import_module("dct_autoencoder.lfq")
    dp = importlib.import_module("dct_autoencoder.dct_patches")
    util = sys.modules["dct_autoencoder.util"]
    return types.SimpleNamespace(fe=fe, patchnorm=pn, lfq=lfq, dct_patches=dp, util=util)
