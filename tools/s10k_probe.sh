#!/bin/bash
# S10k (configs 2/3) probe: per-wave phase clocks (STAMPS build) and the plain bench line.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-s10k}
mkdir -p "$OUT"
JB_LIB=$PWD/exp/stamps/libjiebahip.so JB_STAMPS=1 timeout -k 10 120 python -u bench.py --workload s10k --no-parity \
    --no-e2e --no-profile --steps 3 --warmup 1 > "$OUT/stamps.json" 2> "$OUT/stamps.err"
timeout -k 10 120 python -u bench.py --workload s10k --no-parity --no-e2e --steps 50 --warmup 5 > "$OUT/plain.json" \
    2> "$OUT/plain.err"
grep "\[jb\]" "$OUT/stamps.err" | tail -4 || true
python -c "import json; d=json.load(open('$OUT/plain.json')); print(d['ms_per_step'], d['kernels_ms'])"
