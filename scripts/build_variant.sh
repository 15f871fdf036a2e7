#!/bin/bash
# build a diagnostic variant of libsmg.so with extra compile flags: scripts/build_variant.sh NAME [FLAGS...]
# (SRC=path/to/smg_metrics.hip builds another source of the metrics kernels, e.g. an older revision)
set -e
cd "$(dirname "$0")/../sm_distributed_amd/csrc"
name=$1; shift
src=${SRC:-smg_metrics.hip}
mkdir -p ../variants/$(dirname $name)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I"$PWD" "$@" -c $src -o /tmp/variant_${name//\//_}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread smg_prep.o smg_sort.o smg_isocalc.o smg_rows.o /tmp/variant_${name//\//_}.o -o ../variants/$name.so
echo built variants/$name.so
