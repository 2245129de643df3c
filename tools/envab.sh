#!/bin/bash
# A/B timing of one library under environment settings, REPS rounds interleaved.
# usage: TAG=x REPS=2 tools/envab.sh "JB_ZH_WIDE=0" "JB_ZH_WIDE=1" ...   ("-" = no setting)
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-envab}
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-2}); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    if [ "$e" = "-" ]; then E=""; else E="$e"; fi
    env $E timeout -k 10 300 python bench.py --no-parity --no-e2e --no-latency --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} \
        > "$OUT/v$i.$r.json" 2> "$OUT/v$i.$r.err"
    python -c "import json; d=json.load(open('$OUT/v$i.$r.json')); k=d['kernels_ms']; print('$e', d['ms_per_step'], 'mw', k['k_mark_walk'], 'zh', k['k_zh'], 'nz', k['k_nonzh'])"
  done
done
