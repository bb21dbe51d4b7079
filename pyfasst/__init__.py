"""Drop-in import name: ``import pyfasst.audioModel as am`` (the reference's
own spelling, doc/source/description.rst:50-100) resolves to the MI355X
package ``pyfasst_amd``.

Every ``pyfasst.<name>`` import is served by the SAME module object as
``pyfasst_amd.<name>`` (one class identity, one loaded HIP library), through a
meta-path alias finder; modules the MI355X package does not provide (DEMIX,
NSGT, plotting, ... — out of scope) raise ``ImportError`` as any
missing module would.
"""
import importlib
import importlib.abc
import importlib.util
import sys

_TARGET = "pyfasst_amd"


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target):
        self._target = target

    def create_module(self, spec):
        mod = importlib.import_module(self._target)
        self._spec = mod.__spec__
        return mod

    def exec_module(self, module):
        # already executed under its real name; keep its own spec (the import
        # machinery stamps the alias spec on the shared object)
        module.__spec__ = self._spec


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(__name__ + "."):
            return None
        real = _TARGET + fullname[len(__name__):]
        if importlib.util.find_spec(real) is None:
            return None
        mod = importlib.import_module(real)
        spec = importlib.util.spec_from_loader(
            fullname, _AliasLoader(real), is_package=hasattr(mod, "__path__"))
        return spec


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

_pkg = importlib.import_module(_TARGET)
__version__ = getattr(_pkg, "__version__", None)
