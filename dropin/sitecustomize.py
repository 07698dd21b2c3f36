"""Drop-in switch for the reference's own scripts: `PYTHONPATH=<repo>/dropin`.

With this directory on PYTHONPATH, `import models...` in ANY script resolves to
`deep_prob_feature_track_amd.models` (the HIP-backed mirror of the reference's `models`
package) -- also when the script's own directory holds the reference's `models/` package,
which Python would otherwise find first (the script directory precedes PYTHONPATH on
sys.path).  So the reference's callers run unchanged:

    cd <reference>/code
    PYTHONPATH=<repo>/dropin python evaluate.py ...        # evaluate.py:23-24
    PYTHONPATH=<repo>/dropin python experiments/kf_vo.py   # kf_vo.py:28, select_method.py:8
    PYTHONPATH=<repo>/dropin python convergence_basin.py   # convergence_basin.py:27-28

Python imports `sitecustomize` at start-up from the first sys.path entry that has one; this
one installs a meta-path finder for the names `models` and `models.<sub>`, then runs the
interpreter's own sitecustomize (if any) that it shadows.  Nothing is imported eagerly:
torch and the library load when the script first imports `models`.
"""
import importlib.abc
import importlib.machinery
import importlib.util
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
_TARGET = "deep_prob_feature_track_amd.models"


class _ModelsAlias(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """`models[.sub]` -> the module object of `deep_prob_feature_track_amd.models[.sub]`
    (one module, two names: classes keep their package's __module__, so pickles and
    state_dicts are unaffected)."""

    def find_spec(self, fullname, path=None, target=None):
        if fullname != "models" and not fullname.startswith("models."):
            return None
        real = _TARGET + fullname[len("models"):]
        if importlib.util.find_spec(real) is None:
            return None  # a name the mirror does not provide: ImportError, as for any module
        return importlib.machinery.ModuleSpec(fullname, self, is_package=fullname == "models")

    def create_module(self, spec):
        real = importlib.import_module(_TARGET + spec.name[len("models"):])
        spec._dpft_real_spec = real.__spec__  # restored in exec_module (module_from_spec rebinds it)
        return real

    def exec_module(self, module):
        module.__spec__ = module.__spec__._dpft_real_spec


if _ROOT not in sys.path:
    sys.path.append(_ROOT)
sys.meta_path.insert(0, _ModelsAlias())

# the interpreter's own sitecustomize, which this file shadows
_spec = importlib.machinery.PathFinder.find_spec("sitecustomize", [p for p in sys.path if
                                                                  os.path.abspath(p or ".") != _HERE])
if _spec is not None and _spec.loader is not None:
    _mod = importlib.util.module_from_spec(_spec)
    try:
        _spec.loader.exec_module(_mod)
    except Exception:  # noqa: BLE001 -- a broken site hook must not stop the script
        pass
