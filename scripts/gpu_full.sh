#!/bin/bash
# full session: GPU tests + smoke + bench (+ rocprof stats), then the per-rank shard timing; stops at the first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-full}
bash scripts/gpu_r2.sh $TAG && WS="${WS:-8}" bash scripts/gpu_shards.sh $TAG
