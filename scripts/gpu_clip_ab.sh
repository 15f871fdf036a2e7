#!/bin/bash
# A/B of the clip's ion-stage time over sm_distributed_amd/variants/*.so at 1000x1000 and config 3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-clipab}
mkdir -p gpurun_out/$TAG
for args in "1000 1000 1000 2000 99" "500 500 2000 20000 99"; do
  rm -f gpurun_out/clip_ref.npz
  for so in sm_distributed_amd/variants/*.so; do
    SMG_LIB=$PWD/$so timeout -k 10 300 python3 -u scripts/time_clip.py $args >> gpurun_out/$TAG/clip_ab.txt 2>&1 || exit 1
  done
done
rm -f gpurun_out/clip_ref.npz
grep -v amdgpu gpurun_out/$TAG/clip_ab.txt
