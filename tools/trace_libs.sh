#!/bin/bash
# Kernel durations of several builds of the engine on the same batch, one
# rocprofv3 kernel-trace pass per build (run on the GPU box from the repo root):
#   bash tools/trace_libs.sh TAXA lib1.so lib2.so ...   -> gpurun_out/trace_<lib>/
#   (MODE=nuts for the sampling mode: one call per library)
# then locally: python tools/trace_summary.py gpurun_out/trace_*
set -o pipefail
export TMPDIR=/tmp
taxa=$1; shift
for lib in "$@"; do
  n=$(basename "$lib" .so)
  rm -rf "gpurun_out/trace_$n"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "gpurun_out/trace_$n" -o run --output-format csv -- \
      python3 tools/variant_bench.py "$lib" --reps 1 --steps "${STEPS:-20}" --taxa "$taxa" --mode "${MODE:-map}" \
      > "gpurun_out/trace_$n.log" 2>&1 || exit $?
done
