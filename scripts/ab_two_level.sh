set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/time_metrics.py 2>&1 | grep -v amdgpu && SMG_FORCE_TWO=1 timeout -k 10 300 python scripts/time_metrics.py 2>&1 | grep -v amdgpu
