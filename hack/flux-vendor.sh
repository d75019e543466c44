#!/usr/bin/env bash
# Vendor the pinned Flux release manifest for air-gapped clusters: writes gotk-components.yaml next
# to the remote-URL kustomization and points it at the local file (same version, same content as
# the upstream install.yaml).
set -euo pipefail
cd "$(dirname "$0")/../cluster-config/cluster/flux-system/gotk-components"
ver=$(grep -oE 'releases/download/v[0-9.]+' kustomization.yaml | sed 's#releases/download/##')
if command -v flux >/dev/null; then
  flux install --version="${ver}" --export > gotk-components.yaml
else
  curl -fsSL "https://github.com/fluxcd/flux2/releases/download/${ver}/install.yaml" -o gotk-components.yaml
fi
sed -i "s#  - https://github.com/fluxcd/flux2/releases/download/${ver}/install.yaml#  - gotk-components.yaml#" kustomization.yaml
echo "vendored Flux ${ver}"
