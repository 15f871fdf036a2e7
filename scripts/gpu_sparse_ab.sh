#!/bin/bash
# main-pass A/B at config 3: bench with the sparse main pass (default) and with ion_pipe_kernel<512>
# (--legacy-main), the sparse pass's phase stamps, and a rocprofv3 kernel-stats run.  scripts/gpu_sparse_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-sab}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/bench_sparse.json 2> gpurun_out/$TAG/bench_sparse.err || { tail -30 gpurun_out/$TAG/bench_sparse.err; exit 1; }
tail -2 gpurun_out/$TAG/bench_sparse.err
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_sparse.json'));r=d['roofline'];print('sparse', round(d['ms_per_step'],2),'ms', r['kernel'], round(r['kernel_ms_avg'],2),'ms frac',round(r['frac'],3), d['device_chain']['stages_ms'], d['passes'].get('ion_pipe_kernel<1024> (big-ion LDS pass)'))"
timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --legacy-main > gpurun_out/$TAG/bench_legacy.json 2> gpurun_out/$TAG/bench_legacy.err || { tail -30 gpurun_out/$TAG/bench_legacy.err; exit 1; }
tail -2 gpurun_out/$TAG/bench_legacy.err
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench_legacy.json'));r=d['roofline'];print('legacy', round(d['ms_per_step'],2),'ms', r['kernel'], round(r['kernel_ms_avg'],2),'ms frac',round(r['frac'],3))"
if [ "${STAMPS:-1}" = "1" ]; then
  timeout -k 10 300 python -u scripts/diag_sparse_stamps.py > gpurun_out/$TAG/stamps.txt 2>&1 || { tail -20 gpurun_out/$TAG/stamps.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$TAG/stamps.txt
fi
if [ "${PROFILE:-1}" = "1" ]; then
  rm -rf /tmp/prof_$TAG
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/prof.log 2>&1 || { tail -30 gpurun_out/$TAG/prof.log; exit 1; }
  for f in $(find /tmp/prof_$TAG -name "*kernel_stats.csv"); do cp $f gpurun_out/$TAG/kernel_stats.csv; done
  python3 scripts/short_stats.py gpurun_out/$TAG/kernel_stats.csv | head -12 | tee gpurun_out/$TAG/kernel_stats_short.txt
fi
