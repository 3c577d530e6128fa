#!/bin/bash
# rocprofv3 passes behind profiles/ (run on the GPU box from the repo root):
#   bash tools/profile_round.sh r01      (on the box; then locally:
#   python tools/pmc_summary.py r01 gpurun_out/prof   -> profiles/)
# plus an SQ pass (8 counters: the wave-cycle decomposition) of the C2 bench, and a kernel-trace pass
# and FETCH_SIZE / WRITE_SIZE passes of the NUTS bench (config C3).
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes
# (never combined with trace domains), then the summary.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4-base --no-c3 > "$OUT/bench_trace.json" 2> "$OUT/trace.err" && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c4-base --no-c3 > /dev/null 2> "$OUT/fetch.err" && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c4-base --no-c3 > /dev/null 2> "$OUT/write.err" && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d "$OUT/sq" -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c4-base --no-c3 > /dev/null 2> "$OUT/sq.err" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/nuts_trace" -o run --output-format csv -- \
    python3 bench.py --mode nuts --no-cpu-baseline > "$OUT/bench_nuts_trace.json" 2> "$OUT/nuts_trace.err" && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/nuts_fetch" -o run --output-format csv -- \
    python3 bench.py --mode nuts --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> "$OUT/nuts_fetch.err" && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/nuts_write" -o run --output-format csv -- \
    python3 bench.py --mode nuts --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> "$OUT/nuts_write.err"
