"""Importable alias for the framework package.

The package lives in the directory ``distributed-machine-learning-using-cnn-cifar-10-dataset-_amd/``,
which is not a valid Python identifier.  ``import dmlc`` (and ``import dmlc.<sub>``) resolve to the
modules of that directory *without* creating duplicate module objects: a meta-path finder maps every
``dmlc.X`` name onto the real ``<package>.X`` module, so global state (loaded native libraries,
registered ``torch.ops.dmlc`` operators) exists exactly once.
"""
import importlib
import importlib.abc
import importlib.machinery
import importlib.util
import os
import sys

REAL = "distributed-machine-learning-using-cnn-cifar-10-dataset-_amd"
ALIAS = "dmlc"

_here = os.path.dirname(os.path.abspath(__file__))
if _here not in sys.path:
    sys.path.insert(0, _here)


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, real):
        self.real = real

    def create_module(self, spec):
        return importlib.import_module(self.real)

    def exec_module(self, module):
        pass

    # runpy (``python -m dmlc.<module>``) runs the real module's code object as __main__
    def _real_spec(self):
        return importlib.util.find_spec(self.real)

    def get_code(self, fullname):
        spec = self._real_spec()
        return spec.loader.get_code(self.real)

    def is_package(self, fullname):
        return self._real_spec().submodule_search_locations is not None


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path, target=None):
        if fullname.startswith(ALIAS + "."):
            real = REAL + fullname[len(ALIAS):]
            real_spec = importlib.util.find_spec(real)
            if real_spec is None:
                return None
            spec = importlib.machinery.ModuleSpec(fullname, _AliasLoader(real), origin=real_spec.origin,
                                                  is_package=real_spec.submodule_search_locations is not None)
            spec.has_location = real_spec.has_location
            return spec
        return None


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

sys.modules[ALIAS] = importlib.import_module(REAL)
