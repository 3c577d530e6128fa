#!/bin/bash
# One rocprofv3 SQ-counter pass (the wave-cycle decomposition, 8 counters) over
# tools/variant_bench.py on the given library and batch (run on the GPU box
# from the repo root):
#   bash tools/sq_pass.sh OUT LIB TAXA [MODE]   -> gpurun_out/OUT/
# then locally: python tools/pmc_summary.py-style parsing of the counter CSV.
set -o pipefail
export TMPDIR=/tmp
out=$1 lib=$2 taxa=$3 mode=${4:-map}
rm -rf "gpurun_out/$out"
steps=3
[ "$mode" = nuts ] && steps=1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d "gpurun_out/$out" -o run --output-format csv -- \
    python3 tools/variant_bench.py "$lib" --reps 1 --steps $steps --taxa "$taxa" --mode "$mode" > "gpurun_out/$out.log" 2>&1
