#!/usr/bin/env python3
"""Point a checkout of this repo at YOUR image registry and Git repository.

The tree ships with placeholders (``ghcr.io/example-org/amd-gpu-{operator,bench}`` and
``https://github.com/example-org/k8s-nvidia-gpus_amd.git``).  The reference needs no such step
because every image it names is public (GPU Operator chart, ``cuda-sample:vectoradd``,
``llama.cpp:server-cuda``, ``pytorch/pytorch`` — reference helmrelease.yaml:9-16, README.md:283,
llm/deployment.yaml:61, sd15-api/deployment.yaml:21); here the operator and workload images are
built from this repo and pushed by you (``hack/build-images.sh --registry <yours> --push``; CI's
``images`` job only checks that they build and pushes nothing), so a fresh cluster can only pull
them once the manifests name that registry.

Rewrites, idempotently and re-runnably (the CURRENT values are read from the tree, so running it
again with another registry works):
  * every kustomization ``images:`` ``newName`` and its ``# renovate: depName=`` annotation,
  * the Flux ``GitRepository`` URL (gotk-sync.yaml),
  * Renovate's ``RENOVATE_AUTODISCOVER_FILTER`` (owner/repo of the Git URL),
  * the validator's fallback image (``operator/validator.py``) and the tools' default image,
  * the build comments of the Dockerfiles.

    hack/retarget.py --registry ghcr.io/acme [--git-url https://github.com/acme/k8s-amd.git]
"""
from __future__ import annotations

import argparse
import re
import sys
from pathlib import Path
from typing import Dict, List, Optional, Tuple

REPO = Path(__file__).resolve().parent.parent
OPERATOR_KUSTOMIZATION = "cluster-config/apps/amd-gpu-operator/kustomization.yaml"
GOTK_SYNC = "cluster-config/cluster/flux-system/gotk-sync.yaml"
IMAGE_NAMES = ("amd-gpu-operator", "amd-gpu-bench")


def targets(root: Path) -> List[Path]:
    files = sorted((root / "cluster-config").rglob("*.yaml"))
    files += [root / "k8s_nvidia_gpus_amd/operator/validator.py",
              root / "tools/time_to_first_gpu_pod.py"]
    files += sorted((root / "images").glob("*/Dockerfile"))
    return [f for f in files if f.exists()]


def current_registry(root: Path) -> str:
    text = (root / OPERATOR_KUSTOMIZATION).read_text()
    m = re.search(r"newName:\s*(\S+)/amd-gpu-operator\s*$", text, re.M)
    if not m:
        raise SystemExit(f"no amd-gpu-operator newName in {OPERATOR_KUSTOMIZATION}")
    return m.group(1)


def current_git_url(root: Path) -> str:
    m = re.search(r"^\s*url:\s*(\S+)\s*$", (root / GOTK_SYNC).read_text(), re.M)
    if not m:
        raise SystemExit(f"no GitRepository url in {GOTK_SYNC}")
    return m.group(1)


def owner_repo(git_url: str) -> str:
    m = re.search(r"github\.com[/:]([^/]+)/([^/]+?)(?:\.git)?/?$", git_url)
    if not m:
        raise SystemExit(f"cannot parse owner/repo from {git_url!r} (expected a GitHub URL)")
    return f"{m.group(1)}/{m.group(2)}"


def validate_registry(reg: str) -> str:
    reg = reg.rstrip("/")
    if not re.fullmatch(r"[a-z0-9.\-:]+(/[a-z0-9._\-]+)*", reg):
        raise SystemExit(f"registry {reg!r}: use a lowercase path such as ghcr.io/<owner>")
    return reg


def plan(root: Path, registry: Optional[str], git_url: Optional[str]) -> List[Tuple[str, str]]:
    subs: List[Tuple[str, str]] = []
    if git_url:
        old_url = current_git_url(root)
        subs.append((old_url, git_url))
        subs.append((owner_repo(old_url), owner_repo(git_url)))
    if registry:
        old_reg = current_registry(root)
        for name in IMAGE_NAMES:
            subs.append((f"{old_reg}/{name}", f"{validate_registry(registry)}/{name}"))
    return [(a, b) for a, b in subs if a != b]


def apply(root: Path, registry: Optional[str], git_url: Optional[str],
          dry_run: bool = False) -> Dict[str, int]:
    subs = plan(root, registry, git_url)
    changed: Dict[str, int] = {}
    for f in targets(root):
        text = f.read_text()
        new = text
        n = 0
        for a, b in subs:
            n += new.count(a)
            new = new.replace(a, b)
        if new != text:
            changed[str(f.relative_to(root))] = n
            if not dry_run:
                f.write_text(new)
    return changed


def placeholders_left(root: Path) -> List[str]:
    return [str(f.relative_to(root)) for f in targets(root) if "example-org" in f.read_text()]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--registry", help="image registry prefix, e.g. ghcr.io/acme")
    ap.add_argument("--git-url", help="Git URL Flux pulls, e.g. https://github.com/acme/repo.git")
    ap.add_argument("--root", default=str(REPO))
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--check", action="store_true",
                    help="exit 1 if any example-org placeholder is left (no rewrite)")
    args = ap.parse_args(argv)
    root = Path(args.root)
    if args.check:
        left = placeholders_left(root)
        for f in left:
            print(f"placeholder left: {f}", file=sys.stderr)
        return 1 if left else 0
    if not args.registry and not args.git_url:
        ap.error("nothing to do: pass --registry and/or --git-url")
    changed = apply(root, args.registry, args.git_url, args.dry_run)
    for f, n in changed.items():
        print(f"{'would rewrite' if args.dry_run else 'rewrote'} {f} ({n} substitutions)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
