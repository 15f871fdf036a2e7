#!/bin/bash
# A/B of the variants (scripts/variants.sh), then the round session (scripts/gpu_r2.sh TAG); stops at the first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r2h}
mkdir -p gpurun_out
bash scripts/variants.sh && bash scripts/gpu_r2.sh $TAG
