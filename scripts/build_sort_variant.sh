#!/bin/bash
# build a sort-configuration variant of libsmg.so: scripts/build_sort_variant.sh NAME [FLAGS...]
# (e.g. -DSMG_SRT_IPT=12 -DSMG_SRT_VLOAD=1, csrc/smg_sort.hip's knobs); timed by scripts/time_sort.py with SMG_LIB
set -e
cd "$(dirname "$0")/../sm_distributed_amd/csrc"
name=$1; shift
mkdir -p ../variants/sort
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off "$@" -c smg_sort.hip -o /tmp/sortv_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread smg_prep.o /tmp/sortv_$name.o smg_isocalc.o smg_metrics.o smg_rows.o smg_sparse.o -o ../variants/sort/$name.so
echo built variants/sort/$name.so
