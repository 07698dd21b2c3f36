"""The reference's callers resolve `models.*` against the drop-in with only PYTHONPATH changed.

`dropin/sitecustomize.py` maps `models` / `models.<sub>` onto deep_prob_feature_track_amd.models,
also where the caller's own directory holds the reference's `models/` package (the script
directory precedes PYTHONPATH).  The test reads each caller's import statements (as text,
with `ast`) and resolves them in a child interpreter started in the reference's code
directory -- the situation of `cd code && python evaluate.py` -- checking that every name
binds to this package.  Skipped where the reference tree is absent (the GPU box).
"""
import ast
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_CODE = "/root/reference/code"
CALLERS = ["evaluate.py", "experiments/kf_vo.py", "experiments/select_method.py", "convergence_basin.py",
           "run_example.py"]

needs_ref = pytest.mark.skipif(not os.path.isdir(REF_CODE), reason="reference tree absent")


def _model_imports(path):
    """[(statement kind, module, names / alias)] of the `models` imports in a caller, and the
    attribute names the caller reads from each module alias (`criterions.compute_RPE_loss`)."""
    src = open(path).read()
    out = []
    for node in ast.walk(ast.parse(src)):
        if isinstance(node, ast.Import):
            for a in node.names:
                if a.name == "models" or a.name.startswith("models."):
                    alias = a.asname or a.name
                    attrs = sorted(set(re.findall(rf"\b{re.escape(alias)}\.(\w+)", src)))
                    out.append(("import", a.name, attrs))
        elif isinstance(node, ast.ImportFrom) and node.module and (
                node.module == "models" or node.module.startswith("models.")):
            out.append(("from", node.module, [a.name for a in node.names]))
    return out


_CHILD = r"""
import importlib, json, sys
req = json.loads(sys.argv[1])
res = []
for kind, mod, names in req:
    m = importlib.import_module(mod)
    objs = [getattr(m, n) for n in names]
    res.append([m.__name__] + [getattr(o, "__module__", None) or getattr(o, "__name__", "") for o in objs])
print(json.dumps(res))
"""


@needs_ref
@pytest.mark.parametrize("caller", CALLERS)
def test_reference_caller_resolves_against_dropin(caller):
    req = _model_imports(os.path.join(REF_CODE, caller))
    assert req, f"{caller}: no models imports found"
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "dropin"), PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", _CHILD, json.dumps(req)], cwd=REF_CODE, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for (kind, mod, names), got in zip(req, res):
        assert got[0] == "deep_prob_feature_track_amd." + mod, f"{caller}: {mod} -> {got[0]}"
        for n, owner in zip(names, got[1:]):
            assert owner.startswith("deep_prob_feature_track_amd."), f"{caller}: {mod}.{n} from {owner}"


def test_alias_maps_models_package_without_reference(tmp_path):
    """Also where a shadowing `models/` package sits in the script directory (built here, so
    this runs on any host): the alias wins, the real module keeps its own __spec__."""
    shadow = tmp_path / "models"
    shadow.mkdir()
    (shadow / "__init__.py").write_text("raise ImportError('the shadowed package was imported')\n")
    child = ("import models.LeastSquareTracking as T, models.criterions as C, models; "
             "from models.geometry import batch_create_transform, batch_mat2euler, batch_euler2mat; "
             "assert T.LeastSquareTracking.__module__ == 'deep_prob_feature_track_amd.models.LeastSquareTracking'; "
             "assert T.__spec__.name == 'deep_prob_feature_track_amd.models.LeastSquareTracking', T.__spec__.name; "
             "assert models.__spec__.name == 'deep_prob_feature_track_amd.models'; "
             "assert callable(C.compute_RT_EPE_loss) and callable(C.compute_RPE_loss); print('ok')")
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "dropin"), PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", child], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]
