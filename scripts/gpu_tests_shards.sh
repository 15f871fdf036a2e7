#!/bin/bash
# GPU test suite, then the per-rank shard timing (scripts/gpu_shards.sh); stops at the first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r2j}
BENCH=0 SMOKE=0 bash scripts/gpu_r2.sh $TAG && WS="${WS:-8}" bash scripts/gpu_shards.sh $TAG
