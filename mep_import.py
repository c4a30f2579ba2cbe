"""Register the package directory ``multimodal-emotion-processing_amd/`` (not a valid Python
identifier) as the importable package ``mep_amd``.  Call ``load()`` once; afterwards
``import mep_amd`` and ``from mep_amd import cmu_mosei`` work normally."""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'multimodal-emotion-processing_amd')
NAME = 'mep_amd'


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, '__init__.py'), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules[NAME]
        raise
    return mod
