#!/bin/bash
# Per-wave phase clocks (STAMPS=1 build in exp/stamps) of one bench workload.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-stamps}
mkdir -p "$OUT"
JB_LIB=$PWD/exp/stamps/libjiebahip.so JB_STAMPS=1 timeout -k 10 200 python -u bench.py --no-parity --no-e2e \
    --no-profile --steps 2 --warmup 1 ${BENCH_ARGS:-} > "$OUT/stamps.json" 2> "$OUT/stamps.err"
grep "\[jb\]" "$OUT/stamps.err" | tail -3
