set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/ab_round.sh || exit 1
for so in sm_distributed_amd/variants/sort/*.so; do
  SMG_LIB=$PWD/$so timeout -k 10 300 python scripts/time_sort.py > gpurun_out/sortv.log 2>&1 || { tail -5 gpurun_out/sortv.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/sortv.log
done
