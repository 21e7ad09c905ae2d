"""Import shim: the package directory is ``forest-slam_amd/`` (a hyphenated name Python
cannot import directly).  ``import forest_slam_amd`` from the repo root loads that
directory as the package ``forest_slam_amd``."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_dir = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "forest-slam_amd")
_spec = _ilu.spec_from_file_location("forest_slam_amd", _os.path.join(_dir, "__init__.py"),
                                     submodule_search_locations=[_dir])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["forest_slam_amd"] = _mod
_spec.loader.exec_module(_mod)
