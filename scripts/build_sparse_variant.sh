#!/bin/bash
# a diagnostic variant of libsmg.so whose sparse main pass is built with extra flags:
# scripts/build_sparse_variant.sh NAME [FLAGS...]  -> sm_distributed_amd/variants/NAME.so
set -e
cd "$(dirname "$0")/../sm_distributed_amd/csrc"
name=$1; shift
mkdir -p ../variants
# the library's own flags for this file first (Makefile SPARSE_FLAGS), then the variant's
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I"$PWD" $(make -s print-sparse-flags) "$@" -c smg_sparse.hip -o /tmp/spvariant_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread smg_prep.o smg_sort.o smg_metrics.o smg_isocalc.o smg_rows.o /tmp/spvariant_$name.o -o ../variants/$name.so
echo built variants/$name.so
