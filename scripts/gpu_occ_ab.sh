#!/bin/bash
# occupancy A/B of the main LDS pass: the variants in sm_distributed_amd/variants/ on one workload (VARIANT_ARGS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-occ}
mkdir -p gpurun_out/$TAG
rm -f gpurun_out/variants.log
VARIANT_ARGS="${VARIANT_ARGS:-300 300 2500 20000}" bash scripts/variants.sh || exit 1
cp gpurun_out/variants.log gpurun_out/$TAG/variants.log
