#!/bin/bash
# A/B timing of library variants on config 5b (long-oov): k_long_dp's average per variant.
# usage: tools/ab_long.sh lib name ...   ("lib" = in-tree build, else var/exp_<name>)
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-ablong}
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-1}); do
  for v in "$@"; do
    if [ "$v" = lib ]; then L=$PWD/jieba-go_amd/lib/libjiebahip.so; else L=$PWD/var/exp_$v/libjiebahip.so; fi
    JB_LIB=$L timeout -k 10 300 python bench.py --workload long-oov --no-parity --no-e2e --steps ${STEPS:-3} --warmup 1 \
        > "$OUT/$v.$r.json" 2> "$OUT/$v.$r.err"
    python -c "import json; d=json.load(open('$OUT/$v.$r.json')); k=d['kernels_ms']; print('$v', d['ms_per_step'], {a: round(b, 3) for a, b in k.items() if b > 0.05})"
  done
done
