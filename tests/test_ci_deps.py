"""The CPU CI job installs every third-party module the package and the tests import (VERDICT r4
item 8): a clean ``rocm/dev-ubuntu-22.04`` runner has none of this container's extras, so a hard
import that CI does not install fails there even though every test passes here.

Every ``import`` / ``from … import`` in ``k8s_nvidia_gpus_amd/`` and ``tests/`` (module level or
inside functions) is collected with ``ast``; standard-library and in-repo modules are dropped, as
are optional imports (inside a ``try`` whose handler catches ImportError / Exception, or named in
a ``pytest.importorskip``).  What remains must map to a package the CI job's ``pip3 install``
lines name."""
import ast
import re
import sys
from pathlib import Path

import yaml

REPO = Path(__file__).resolve().parent.parent
# import name -> pip distribution (when they differ); modules that come with another package
PIP_NAME = {"yaml": "pyyaml", "grpc": "grpcio", "google": "protobuf", "PIL": "pillow",
            "starlette": "fastapi", "pydantic": "fastapi", "anyio": "fastapi"}
LOCAL = {"k8s_nvidia_gpus_amd", "fakes", "tests", "conftest", "__graft_entry__"}
# not pip packages of the CPU job: imported lazily only on the nodes / images that have them, and
# the CPU tests drive fakes in their place
RUNTIME_PROVIDED = {"amdsmi": "ROCm's amd-smi Python bindings (operator image; tests: fakes/amdsmi)",
                    "diffusers": "the diffusers A/B backend of the SD1.5 API (serving image only)"}


def _optional_nodes(tree):
    """Import nodes inside a try whose handlers catch ImportError / Exception / everything."""
    out = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Try):
            names = set()
            for h in node.handlers:
                t = h.type
                for e in (t.elts if isinstance(t, ast.Tuple) else [t]):
                    names.add(getattr(e, "id", None) if e is not None else "*")
            if names & {"ImportError", "ModuleNotFoundError", "Exception", "*", "BaseException"}:
                for b in node.body:
                    for sub in ast.walk(b):
                        if isinstance(sub, (ast.Import, ast.ImportFrom)):
                            out.add(id(sub))
    return out


def third_party_imports():
    stdlib = set(sys.stdlib_module_names)
    found = {}
    files = list((REPO / "k8s_nvidia_gpus_amd").rglob("*.py")) + list((REPO / "tests").rglob("*.py"))
    for f in files:
        src = f.read_text()
        tree = ast.parse(src)
        optional = _optional_nodes(tree)
        skipped = set(re.findall(r"importorskip\(\s*[\"']([\w.]+)", src))
        for node in ast.walk(tree):
            if isinstance(node, ast.Import):
                mods = [a.name for a in node.names]
            elif isinstance(node, ast.ImportFrom) and node.level == 0 and node.module:
                mods = [node.module]
            else:
                continue
            if id(node) in optional:
                continue
            for m in mods:
                top = m.split(".")[0]
                if top in stdlib or top in LOCAL or top.startswith("test_") or m in skipped \
                        or top in skipped or top in RUNTIME_PROVIDED:
                    continue
                found.setdefault(top, set()).add(str(f.relative_to(REPO)))
    return found


def ci_packages():
    ci = yaml.safe_load((REPO / ".github/workflows/ci.yaml").read_text())
    pkgs = set()
    for step in ci["jobs"]["cpu"]["steps"]:
        run = step.get("run", "")
        for line in run.replace("\\\n", " ").splitlines():
            if "pip3 install" in line:
                words = line.split("pip3 install", 1)[1].split()
                pkgs |= {w.lower() for w in words if not w.startswith("-") and "://" not in w}
    return pkgs


def test_every_third_party_import_is_installed_by_ci():
    pkgs = ci_packages()
    assert "torch" in pkgs and "pytest" in pkgs
    missing = {}
    for mod, where in sorted(third_party_imports().items()):
        pip = PIP_NAME.get(mod, mod).lower()
        if pip not in pkgs:
            missing[mod] = sorted(where)[:3]
    assert not missing, f"imported but not installed by .github/workflows/ci.yaml: {missing}"
