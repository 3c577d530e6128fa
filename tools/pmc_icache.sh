#!/bin/bash
# Instruction-cache counters of the MAP call, one rocprofv3 --pmc pass per
# build (development): tools/pmc_icache.sh [TAXA] [LIB.so ...]
#   -> gpurun_out/ic_<lib>/run_counter_collection.csv
set -e
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
taxa=${1:-10000}; shift || true
libs=("$@"); [ ${#libs[@]} -eq 0 ] && libs=(metadamage_amd/libmdfit.so)
for lib in "${libs[@]}"; do
  v=$(basename "$lib" .so)
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
    -d gpurun_out/ic_$v -o run --output-format csv -- python3 tools/prof_split.py "$taxa" "$lib" > gpurun_out/ic_$v.log 2>&1
done
