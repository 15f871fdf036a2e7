#!/bin/bash
# build a diagnostic variant of libsmg.so with extra compile flags: scripts/build_variant.sh NAME [FLAGS...]
set -e
cd "$(dirname "$0")/../sm_distributed_amd/csrc"
name=$1; shift
mkdir -p ../variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off "$@" -c smg_metrics.hip -o /tmp/variant_${name//\//_}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC smg_prep.o /tmp/variant_${name//\//_}.o -o ../variants/$name.so
echo built variants/$name.so
