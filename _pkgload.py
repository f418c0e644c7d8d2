"""Registers the product package directory (whose name is not a Python
identifier) under the import name ``midiseq``."""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "deep-learning-based-sequence-models-for-music-generation_amd")


def load():
    if "midiseq" in sys.modules:
        return sys.modules["midiseq"]
    spec = importlib.util.spec_from_file_location(
        "midiseq", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["midiseq"] = mod
    spec.loader.exec_module(mod)
    return mod
