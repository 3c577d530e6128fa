#!/bin/bash
# Build a variant of libmdfit.so with extra compile flags (development A/B):
#   tools/build_variant.sh NAME -DFLAG=1 ...  ->  metadamage_amd/libmdfit_NAME.so
# The library's two translation units as in __graft_entry__.build_hip; the
# flags given apply to both, MAP_FLAGS / NUTS_FLAGS (environment) to one unit
# only (mdfit.hip / mdfit_nuts.hip; NUTS_FLAGS defaults to the product's
# -disable-machine-licm).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result"
NUTS_FLAGS=${NUTS_FLAGS--mllvm -disable-machine-licm}
$H "$@" $MAP_FLAGS -c "$ROOT/metadamage_amd/csrc/mdfit.hip" -o "$tmp/mdfit.o" &
$H "$@" $NUTS_FLAGS -c "$ROOT/metadamage_amd/csrc/mdfit_nuts.hip" -o "$tmp/mdfit_nuts.o" &
wait %1 && wait %2
$H -shared "$tmp/mdfit.o" "$tmp/mdfit_nuts.o" -o "$ROOT/metadamage_amd/libmdfit_$name.so"
