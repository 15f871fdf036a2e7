#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-rX}
bash scripts/gpu_round_diag.sh $TAG && bash scripts/gpu_pmc.sh $TAG
