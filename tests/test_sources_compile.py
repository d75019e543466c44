"""Every Python source of the package, the tools and the entry points byte-compiles (a syntax error
in a GPU-only module would otherwise surface only on the GPU box)."""
import pathlib
import py_compile

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
SOURCES = sorted([*ROOT.glob("k8s_nvidia_gpus_amd/**/*.py"), *ROOT.glob("tools/**/*.py"),
                  *ROOT.glob("hack/*.py"), *ROOT.glob("scripts/*.py"), ROOT / "bench.py",
                  ROOT / "__graft_entry__.py"])


@pytest.mark.parametrize("path", SOURCES, ids=lambda p: str(p.relative_to(ROOT)))
def test_source_compiles(path, tmp_path):
    py_compile.compile(str(path), cfile=str(tmp_path / "x.pyc"), doraise=True)
