#!/bin/bash
# The other BASELINE.json configs as bench lines (config 4, the headline, is bench.py's default).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-cfg}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  echo "== $name"
  timeout -k 10 300 python bench.py --no-e2e "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  python -c "import json; d=json.load(open('$OUT/$name.json')); c=d['cpu_baseline'] or {}; print('$name', d['ms_per_step'], 'ms', round(d['value']/1e9,3), 'G chars/s', 'cpu', c.get('value'), 'parity', (d['parity'] or {}).get('bit_exact'))"
}
echo "== sentence"
timeout -k 10 300 python bench.py --workload sentence > "$OUT/sentence.json" 2> "$OUT/sentence.err"
tail -c 600 "$OUT/sentence.json"; echo
run s10k_hmm0 --workload s10k --hmm 0
run s10k_hmm1 --workload s10k --hmm 1
run l1m_punct --workload long-punct --steps 5 --warmup 2
run l1m_oov --workload long-oov --steps 3 --warmup 1
echo "== done"
