#!/bin/bash
# Build libmdfit_NAME.so from the sources of git revision REV (development A/B):
#   tools/build_ref_variant.sh NAME REV [-DFLAG=1 ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=$2; shift 2
tmp=$(mktemp -d)
mkdir -p "$tmp/include" "$tmp/metadamage_amd/csrc"
for f in include/mdfit.h metadamage_amd/csrc/mdfit.hip metadamage_amd/csrc/mdfit_nuts.hip \
         metadamage_amd/csrc/mdfit_special.h metadamage_amd/csrc/mdfit_model.h metadamage_amd/csrc/mdfit_host.h; do
  git -C "$ROOT" show "$rev:$f" > "$tmp/$f"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result "$@" \
  "$tmp/metadamage_amd/csrc/mdfit.hip" "$tmp/metadamage_amd/csrc/mdfit_nuts.hip" \
  -o "$ROOT/metadamage_amd/libmdfit_$name.so"
rm -rf "$tmp"
