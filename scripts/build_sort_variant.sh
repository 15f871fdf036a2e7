#!/bin/bash
# build a sort-configuration variant of libsmg.so: scripts/build_sort_variant.sh NAME [FLAGS...]
# (e.g. -DSMG_SORT_RADIX_BITS=9 -DSMG_SORT_BLOCK=512 -DSMG_SORT_IPT=16); timed by scripts/sort_ab.sh
set -e
cd "$(dirname "$0")/../sm_distributed_amd/csrc"
name=$1; shift
mkdir -p ../variants/sort
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off "$@" -c smg_prep.hip -o /tmp/sortv_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread /tmp/sortv_$name.o smg_isocalc.o smg_metrics.o -o ../variants/sort/$name.so
echo built variants/sort/$name.so
