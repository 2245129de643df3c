#!/bin/bash
# Round-end evidence on one GPU: PMC passes (headline workload) -> PMC summary,
# rocprofv3 kernel stats of the bench, then the full default bench line (which
# reads the PMC summary for roofline.traffic).  usage: TAG=r02d tools/final_profile.sh
set -euo pipefail
cd "$(dirname "$0")/.."
T=${TAG:-final}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=$T/pmc tools/pmc.sh
python3 tools/pmc_summary.py "$OUT/pmc" "$OUT/pmc_latest.json" "1 GiB C_syn corpus, prefix dict, hmm on; $T"
cp "$OUT/pmc_latest.json" profiles/pmc_latest.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
    python3 bench.py --no-parity --no-e2e --no-latency --steps 10 --warmup 3 > "$OUT/stats_bench.json" 2> "$OUT/stats_bench.err"
timeout -k 10 500 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
tail -1 "$OUT/bench.json"
