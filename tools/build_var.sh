#!/bin/bash
# Build a variant engine library with compile-time KD options for A/B timing:
#   tools/build_var.sh <name> "-DKD_WDYN=1 -DKD_SDIV=8"  ->  shadow_amd/libshd_route_<name>.so
# then: bash tools/gpu_ab4.sh "SHD_ROUTE_LIB=shadow_amd/libshd_route_<name>.so"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
shift
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-result \
  $* -o "$ROOT/shadow_amd/libshd_route_$NAME.so" "$ROOT/shadow_amd/csrc/engine.hip"
echo "built shadow_amd/libshd_route_$NAME.so"
