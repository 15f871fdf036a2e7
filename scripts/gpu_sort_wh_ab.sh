#!/bin/bash
# sort count-kernel A/B: per-wave histograms (current build) vs one histogram per tile (variant), scripts/time_sort.py
# alternating, then the sort tests on the current build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-swh}
mkdir -p gpurun_out/$TAG
for r in new1 old1 new2 old2; do
  case $r in old*) L=sm_distributed_amd/variants/sort/nowh.so;; *) L=sm_distributed_amd/libsmg.so;; esac
  timeout -k 10 300 env SMG_LIB=$L python3 -u scripts/time_sort.py > gpurun_out/$TAG/$r.txt 2>&1 || { tail -20 gpurun_out/$TAG/$r.txt; exit 1; }
  echo "$r: $(grep -E 'fused flag_and_sort +min|hand-written sort alone' gpurun_out/$TAG/$r.txt | tr '\n' ' ')"
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sort.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1; tail -2 gpurun_out/$TAG/pytest.log
