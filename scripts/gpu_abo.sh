#!/bin/bash
# oracle arbitration between library variants (scripts/ab_oracle.py):
#   scripts/gpu_abo.sh TAG name:variant ...   (variant = sm_distributed_amd/variants/<variant>.so, or "lib" = libsmg.so)
# saves each name's table, then checks every later name against the first (differences -> oracle);
# then the phase stamps when libsmg_stamps.so is present
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
names=()
for nv in "$@"; do
  n=${nv%%:*}; v=${nv#*:}
  if [ "$v" = lib ]; then L=$PWD/sm_distributed_amd/libsmg.so; else L=$PWD/sm_distributed_amd/variants/$v.so; fi
  SMG_LIB=$L timeout -k 10 300 python3 -u scripts/ab_oracle.py save $n >> gpurun_out/$TAG/abo.txt 2>&1 || exit 1
  names+=($n)
done
for n in "${names[@]:1}"; do
  echo "## ${names[0]} vs $n" >> gpurun_out/$TAG/abo.txt
  timeout -k 10 600 python3 -u scripts/ab_oracle.py check ${names[0]} $n >> gpurun_out/$TAG/abo.txt 2>&1 || exit 1
done
if [ -f sm_distributed_amd/libsmg_stamps.so ]; then
  timeout -k 10 300 python3 -u scripts/diag_stamps.py > gpurun_out/$TAG/stamps.txt 2>&1 || exit 1
fi
