#!/bin/bash
# A/B timing of library variants on the GPU box: bench.py (no CPU leg) per
# variant, REPS rounds interleaved.  usage: tools/abtest.sh lib lib_name ...
# ("lib" = the in-tree jieba-go_amd/lib build, else var/exp_<name>).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    if [ "$v" = lib ]; then L=$PWD/jieba-go_amd/lib/libjiebahip.so; else L=$PWD/var/exp_$v/libjiebahip.so; fi
    JB_LIB=$L timeout -k 10 300 python bench.py --no-parity --no-e2e --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} \
        > "$OUT/$v.$r.json" 2> "$OUT/$v.$r.err"
    python -c "import json; d=json.load(open('$OUT/$v.$r.json')); k=d['kernels_ms']; print('$v', d['ms_per_step'], 'mw', k['k_mark_walk'], 'zh', k['k_zh'], 'nz', k['k_nonzh'])"
  done
done
