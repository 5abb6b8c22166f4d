"""Load ``fish-eye_bundle_adjustment_amd/`` (a hyphenated directory) as the package ``fba_amd``."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "fish-eye_bundle_adjustment_amd")


def load():
    if "fba_amd" in sys.modules:
        return sys.modules["fba_amd"]
    spec = importlib.util.spec_from_file_location("fba_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["fba_amd"] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules["fba_amd"]
        raise
    return mod
