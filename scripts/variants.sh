#!/bin/bash
# A/B timing of sm_distributed_amd/variants/*.so (diagnostic builds of the same C-ABI), in name order, one
# process each; the first is the reference the others are compared with (scripts/time_metrics.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/ab_ref.npz
# a kept reference table (abref/ab_ref.npz, e.g. from an earlier library with another ABI) replaces the first variant
[ -f abref/ab_ref.npz ] && cp abref/ab_ref.npz gpurun_out/ab_ref.npz
for so in sm_distributed_amd/variants/*.so; do
  SMG_LIB=$PWD/$so timeout -k 10 300 python scripts/time_metrics.py ${VARIANT_ARGS} > gpurun_out/variant.log 2>&1
  rc=$?
  grep -v amdgpu.ids gpurun_out/variant.log | tee -a gpurun_out/variants.log
  [ $rc -eq 0 ] || exit $rc
done
