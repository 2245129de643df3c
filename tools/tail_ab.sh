#!/bin/bash
# k_zh tail groups: per-wave totals (STAMPS build) and A/B timing of JB_ZH_TAIL_KIB /
# JB_ZH_TAIL_GROUP settings, then one full-parity bench under the last setting.
# usage: TAG=tail1 tools/tail_ab.sh "JB_ZH_TAIL_KIB=0" "JB_ZH_TAIL_KIB=32768 JB_ZH_TAIL_GROUP=1024" ...
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-tail}
mkdir -p "$OUT"
i=0
for v in "$@"; do
  i=$((i+1))
  env $v JB_LIB=$PWD/jieba-go_amd/lib_st/libjiebahip.so JB_STAMPS=1 timeout -k 10 200 python -u bench.py --no-parity \
      --no-e2e --no-profile --no-latency --steps 2 --warmup 1 > "$OUT/st$i.json" 2> "$OUT/st$i.err"
  echo "$v: $(grep 'wave totals' "$OUT/st$i.err" | tail -1)"
done
TAG=${TAG:-tail}/ab tools/envab.sh "$@"
last="${!#}"
env $last timeout -k 10 300 python -u bench.py --no-e2e --no-latency --steps 10 --warmup 3 > "$OUT/parity.json" 2> "$OUT/parity.err"
python -c "import json; d=json.load(open('$OUT/parity.json')); print('parity', d.get('parity'), d['ms_per_step'])"
