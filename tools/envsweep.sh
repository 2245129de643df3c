#!/bin/bash
# Bench variants selected by environment knobs, each with a parity sample.
# SPECS="JB_ZH_GRP=1 JB_ZH_GRP=4,JB_GRID_ZH=8192"  (comma joins variables of one run)
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-sweep}
mkdir -p "$OUT"
i=0
for spec in ${SPECS:-"JB_ZH_GRP=1"}; do
  i=$((i+1))
  echo "== $spec"
  env ${spec//,/ } JB_DEBUG=1 timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --cpu-sample-mib ${PAR_MIB:-16} \
      ${BENCH_ARGS:-} > "$OUT/s$i.json" 2> "$OUT/s$i.err"
  python -c "import json; d=json.load(open('$OUT/s$i.json')); print(d['ms_per_step'], d['parity_sample']['bit_exact'], d['kernels_ms'])"
  grep "\[jb\]" "$OUT/s$i.err" | tail -1
done
