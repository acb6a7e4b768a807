"""Import helper: the package lives in the directory ``dct-autoencoder_amd/``
(a name Python cannot import directly); this registers it as the module
``dct_autoencoder_amd``."""
import importlib.util
import os
import sys

NAME = "dct_autoencoder_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dct-autoencoder_amd")


def load():
    mod = sys.modules.get(NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop(NAME, None)
        raise
    return mod
