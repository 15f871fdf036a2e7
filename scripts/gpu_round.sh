#!/bin/bash
# tests then bench+profile, stop at first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-rX}
bash scripts/gpu_tests.sh && bash scripts/gpu_bench.sh $TAG
