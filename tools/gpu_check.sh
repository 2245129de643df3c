#!/bin/bash
# One GPU session: smoke -> parity tests -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== smoke" && timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1
echo "== pytest -m gpu" && timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
echo "== bench" && timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
if [ "${PROF:-1}" = "1" ]; then
  echo "== rocprofv3"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
fi
echo "== done"
