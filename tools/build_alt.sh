#!/bin/bash
# Build an alternative engine library for A/B timing:
#   tools/build_alt.sh <file> <header-name-it-replaces> [name]
# e.g. tools/build_alt.sh /tmp/sssp_delta_old.hpp sssp_delta.hpp  ->  shadow_amd/libshd_route_alt.so
# then: bash tools/gpu_ab.sh "" "SHD_ROUTE_LIB=shadow_amd/libshd_route_alt.so"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SUB=$1
HDR=$2
NAME=${3:-alt}
TMP=$(mktemp -d)
mkdir -p "$TMP/a/b"
cp -r "$ROOT/shadow_amd/csrc" "$TMP/a/b/csrc"
cp -r "$ROOT/include" "$TMP/a/include"
cp "$SUB" "$TMP/a/b/csrc/$HDR"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-result \
  -I"$ROOT/include" -o "$ROOT/shadow_amd/libshd_route_$NAME.so" "$TMP/a/b/csrc/engine.hip"
rm -rf "$TMP"
echo "built shadow_amd/libshd_route_$NAME.so"
