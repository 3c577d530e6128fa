#!/bin/bash
# Build a variant of libmdfit.so with extra compile flags (development A/B):
#   tools/build_variant.sh NAME -DFLAG=1 ...  ->  metadamage_amd/libmdfit_NAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result "$@" \
  "$ROOT/metadamage_amd/csrc/mdfit.hip" "$ROOT/metadamage_amd/csrc/mdfit_nuts.hip" \
  -o "$ROOT/metadamage_amd/libmdfit_$name.so"
