#!/usr/bin/env bash
# Build the operator and bench/workload images for a registry you own, and (only with --push)
# push them; then `hack/bootstrap.sh --registry <prefix>` points the GitOps tree at them.
#   hack/build-images.sh --registry ghcr.io/<you> [--tag 0.1.0] [--push]
set -euo pipefail
cd "$(dirname "$0")/.."
REGISTRY="" TAG="0.1.0" PUSH=0
while [[ $# -gt 0 ]]; do
  case "$1" in
    --registry) REGISTRY="$2"; shift 2 ;;
    --tag) TAG="$2"; shift 2 ;;
    --push) PUSH=1; shift ;;
    *) echo "unknown argument: $1" >&2; exit 2 ;;
  esac
done
[[ -n "$REGISTRY" ]] || { echo "usage: $0 --registry <registry/prefix> [--tag T] [--push]" >&2; exit 2; }
[[ "$REGISTRY" == *example-org* ]] && { echo "refusing the example-org placeholder" >&2; exit 2; }
for img in operator bench; do
  ref="${REGISTRY%/}/amd-gpu-${img}:${TAG}"
  docker build -f "images/${img}/Dockerfile" -t "$ref" .
  if [[ $PUSH == 1 ]]; then docker push "$ref"; fi
  echo "$ref"
done
