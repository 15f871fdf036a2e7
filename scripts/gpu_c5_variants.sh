#!/bin/bash
# Config-5 rank-0 shard (scripts/time_shards.py, ONLY_RANK=0) for libsmg.so and every sm_distributed_amd/variants/*.so:
# the wide pass's HIP-event time per library -> gpurun_out/$TAG/c5_<lib>.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-c5v}
mkdir -p gpurun_out/$TAG
for so in sm_distributed_amd/libsmg.so $(ls sm_distributed_amd/variants/*.so 2>/dev/null); do
  n=$(basename $so .so)
  SMG_LIB=$PWD/$so CONFIG=5 SKIP_T1=1 ONLY_RANK=0 timeout -k 10 400 python3 -u scripts/time_shards.py 8 \
    > gpurun_out/$TAG/c5_$n.txt 2>&1 || { tail -20 gpurun_out/$TAG/c5_$n.txt; exit 1; }
  echo "$n: $(grep -o 'wide pass[^;]*ms' gpurun_out/$TAG/c5_$n.txt | head -1)"
done
