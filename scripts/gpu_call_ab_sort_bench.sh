set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/sort_ab.sh || exit 1
mkdir -p gpurun_out/r18
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r18/bench.json 2> gpurun_out/r18/bench.err || { tail -20 gpurun_out/r18/bench.err; exit 1; }
cat gpurun_out/r18/bench.json
