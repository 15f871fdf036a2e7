#!/bin/bash
# phase stamps at 300x300 px (where ion_pipe_kernel fits four 256-thread workgroups per CU): the sparse pass
# (libsmg_stamps.so) against ion_pipe_kernel<256> x 4 (libsmg_stamps256.so), then the sparse pass at config 3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-scmp}
mkdir -p gpurun_out/$TAG
W="300 300 2500 20000"
timeout -k 10 300 python -u scripts/diag_sparse_stamps.py $W > gpurun_out/$TAG/sparse_300.txt 2>&1 || { tail -20 gpurun_out/$TAG/sparse_300.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/sparse_300.txt
SMG_LIB=$PWD/sm_distributed_amd/libsmg_stamps256.so timeout -k 10 300 python -u scripts/diag_stamps.py $W > gpurun_out/$TAG/legacy256_300.txt 2>&1 || { tail -20 gpurun_out/$TAG/legacy256_300.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/legacy256_300.txt
timeout -k 10 300 python -u scripts/diag_sparse_stamps.py > gpurun_out/$TAG/sparse_c3.txt 2>&1 || { tail -20 gpurun_out/$TAG/sparse_c3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/sparse_c3.txt
