#!/usr/bin/env bash
# Bootstrap Flux on a fresh RKE2 cluster (the reference's README.md:248-262 steps, scripted).
#   hack/bootstrap.sh [--git-url https://github.com/<you>/k8s-nvidia-gpus_amd.git]
# Needs kubectl pointing at the cluster (ansible-playbook ... fetch-kubeconfig.yaml) and
# GITHUB_TOKEN (direnv / .envrc).
set -euo pipefail
cd "$(dirname "$0")/.."
GIT_URL=""
while [[ $# -gt 0 ]]; do
  case "$1" in
    --git-url) GIT_URL="$2"; shift 2 ;;
    *) echo "unknown arg $1" >&2; exit 2 ;;
  esac
done
: "${GITHUB_TOKEN:?export GITHUB_TOKEN (see .envrc)}"
if [[ -n "$GIT_URL" ]]; then
  sed -i "s#^\(  url: \).*#\1${GIT_URL}#" cluster-config/cluster/flux-system/gotk-sync.yaml
fi
start=$(date +%s)
kubectl create namespace flux-system --dry-run=client -o yaml | kubectl apply -f -
kubectl -n flux-system create secret generic flux-system \
  --from-literal=username=git --from-literal=password="${GITHUB_TOKEN}" \
  --dry-run=client -o yaml | kubectl apply -f -
kubectl apply -k cluster-config/cluster/flux-system/
echo "waiting for Flux to reconcile the AMD GPU operator..."
kubectl -n flux-system wait kustomization/amd-gpu-operator --for=condition=Ready --timeout=30m
python3 tools/time_to_first_gpu_pod.py --since "$start"
