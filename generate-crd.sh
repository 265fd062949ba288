#!/usr/bin/env bash
# Regenerates the chart's CRD from the native crdgen (reference generate-crd.sh:7).
set -euo pipefail
cd "$(dirname "$0")"
python3 -m bacchus_gpu_controller_amd.utils.build >/dev/null
./bin/crdgen > ./charts/bacchus-gpu-controller/templates/crd.yaml
