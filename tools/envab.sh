#!/bin/bash
# A/B of environment settings with the in-tree library: bench.py (no CPU leg)
# per setting, REPS rounds interleaved.  usage: tools/envab.sh "JB_X=0" "JB_X=1" ...
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-envab}
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-2}); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 300 python bench.py --no-parity --no-e2e --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} \
        > "$OUT/v$i.$r.json" 2> "$OUT/v$i.$r.err"
    python -c "import json; d=json.load(open('$OUT/v$i.$r.json')); k=d['kernels_ms']; print('$v', d['ms_per_step'], 'mw', k['k_mark_walk'], 'zh', k['k_zh'], 'nz', k['k_nonzh'])"
  done
done
