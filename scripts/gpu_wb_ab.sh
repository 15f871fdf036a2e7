#!/bin/bash
# window search A/B: the cooperative kernel (current build) vs the per-lane one (variant), identical outputs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-wb}
mkdir -p gpurun_out/$TAG
for r in new old new2 old2; do
  case $r in old*) L=sm_distributed_amd/variants/wb0.so;; *) L=sm_distributed_amd/libsmg.so;; esac
  timeout -k 10 300 env SMG_LIB=$L python3 -u scripts/time_window_bounds.py /tmp/wb_$r.npz 2>&1 | grep -v amdgpu.ids || exit 1
done
python3 -c "
import numpy as np
a=np.load('/tmp/wb_new.npz'); b=np.load('/tmp/wb_old.npz')
print('identical:', all(np.array_equal(a[k], b[k]) for k in ('lo','hi','lo2','hi2')))
"
