#!/bin/bash
# main-pass A/B over library builds (variants/*.so vs libsmg.so), alternating, with a bit-for-bit table check
cd "${GRAFT_REPO_ROOT:-/root/repo}"
LIBS="sm_distributed_amd/libsmg.so $(ls sm_distributed_amd/variants/*.so)"
for round in 1 2; do
  for L in $LIBS; do
    b=$(basename $L .so)
    timeout -k 10 300 env SMG_LIB=$L python3 -u scripts/ab_libs.py /tmp/ab_$b.npz 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
python3 -c "
import numpy as np, glob
base = np.load('/tmp/ab_libsmg.npz')['vals']
for f in sorted(glob.glob('/tmp/ab_*.npz')):
    v = np.load(f)['vals']
    print(f, 'identical' if v.shape == base.shape and np.array_equal(v, base) else 'max|d| %.3g' % np.abs(v - base).max())
"
