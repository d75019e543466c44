"""Copy in-package app sources into the Kustomize trees that ship them as ConfigMaps.

Kustomize's configMapGenerator only reads files inside the kustomization directory, so the SD1.5
service (k8s_nvidia_gpus_amd/models/sd15_api.py) is mirrored to cluster-config/apps/sd15-api/app/
app.py.  tests/test_static_manifests.py fails when the two drift.

    python -m k8s_nvidia_gpus_amd.utils.sync_apps [--check]
"""
from __future__ import annotations

import argparse
import shutil
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
PAIRS = [
    (REPO / "k8s_nvidia_gpus_amd/models/sd15_api.py", REPO / "cluster-config/apps/sd15-api/app/app.py"),
]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args(argv)
    drift = [dst for src, dst in PAIRS if not dst.exists() or dst.read_bytes() != src.read_bytes()]
    if args.check:
        for d in drift:
            print(f"out of sync: {d.relative_to(REPO)}")
        return 1 if drift else 0
    for src, dst in PAIRS:
        shutil.copyfile(src, dst)
    return 0


if __name__ == "__main__":
    sys.exit(main())
