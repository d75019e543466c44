#!/usr/bin/env bash
# Bootstrap Flux on a fresh RKE2 cluster (the reference's README.md:248-262 steps, scripted).
#   hack/bootstrap.sh --registry <registry-prefix> [--git-url https://github.com/<you>/k8s-nvidia-gpus_amd.git]
# --registry points every operator/workload image at the registry you pushed the images to
# (images/{operator,bench}/Dockerfile; hack/build-images.sh); --git-url is the repo Flux pulls.
# Both rewrite the checkout (hack/retarget.py) — commit and push the result so Flux sees it.
# Needs kubectl pointing at the cluster (ansible-playbook ... fetch-kubeconfig.yaml) and
# GITHUB_TOKEN (direnv / .envrc).
set -euo pipefail
cd "$(dirname "$0")/.."
GIT_URL=""
REGISTRY=""
while [[ $# -gt 0 ]]; do
  case "$1" in
    --git-url) GIT_URL="$2"; shift 2 ;;
    --registry) REGISTRY="$2"; shift 2 ;;
    *) echo "unknown arg $1" >&2; exit 2 ;;
  esac
done
args=()
[[ -n "$REGISTRY" ]] && args+=(--registry "$REGISTRY")
[[ -n "$GIT_URL" ]] && args+=(--git-url "$GIT_URL")
if [[ ${#args[@]} -gt 0 ]]; then
  python3 hack/retarget.py "${args[@]}"
fi
# placeholder images never exist: every DaemonSet would sit in ImagePullBackOff and the
# amd-gpu-operator Kustomization (wait: true) would never turn Ready
if ! python3 hack/retarget.py --check; then
  echo "example-org placeholders left: pass --registry <your registry> --git-url <your fork>" >&2
  exit 2
fi
if ! git diff --quiet -- cluster-config 2>/dev/null; then
  echo "note: cluster-config was rewritten; commit and push it before Flux reconciles" >&2
fi
: "${GITHUB_TOKEN:?export GITHUB_TOKEN (see .envrc)}"
start=$(date +%s)
kubectl create namespace flux-system --dry-run=client -o yaml | kubectl apply -f -
kubectl -n flux-system create secret generic flux-system \
  --from-literal=username=git --from-literal=password="${GITHUB_TOKEN}" \
  --dry-run=client -o yaml | kubectl apply -f -
kubectl apply -k cluster-config/cluster/flux-system/
echo "waiting for Flux to reconcile the AMD GPU operator..."
kubectl -n flux-system wait kustomization/amd-gpu-operator --for=condition=Ready --timeout=30m
python3 tools/time_to_first_gpu_pod.py --since "$start"
