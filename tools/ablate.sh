#!/bin/bash
# Diagnostic ablations (timings only; outputs are wrong under JB_ABLATE != 0).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-abl}
mkdir -p "$OUT"
for cfg in ${CFGS:-"0:0" "1:0" "2:0" "4:0" "0:8192" "0:65536"}; do
  a=${cfg%%:*}; g=${cfg##*:}
  echo "== ablate=$a grid=$g"
  JB_DEBUG=1 JB_ABLATE=$a JB_GRID_ZH=$g timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 2 ${BENCH_ARGS:-} > "$OUT/a${a}_g${g}.json" 2> "$OUT/a${a}_g${g}.err"
  python -c "import json,sys; d=json.load(open('$OUT/a${a}_g${g}.json')); print(d['ms_per_step'], d['kernels_ms'])"
  grep "\[jb\]" "$OUT/a${a}_g${g}.err" | tail -1
done
