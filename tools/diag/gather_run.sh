#!/bin/bash
# gather microbenchmark on one GPU: plain timings, then two PMC passes (L1 accesses,
# TA/TD busy) over a shorter run of the same configurations.  usage: RUN=r04b bash tools/diag/gather_run.sh
set -euo pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${RUN:-gather}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 tools/diag/gather 512 > "$OUT/gather.jsonl"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d "$OUT/pmc1" -o run --output-format csv -- tools/diag/gather 128 > "$OUT/gather_p1.jsonl" 2> "$OUT/p1.err"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE -d "$OUT/pmc2" -o run --output-format csv -- tools/diag/gather 128 > "$OUT/gather_p2.jsonl" 2> "$OUT/p2.err"
echo done
