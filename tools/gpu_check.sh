#!/bin/bash
# One GPU session: smoke -> parity tests -> bench (+ variants) -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${SMOKE:-1}" = "1" ]; then
  echo "== smoke" && timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1
fi
if [ "${TESTS:-1}" = "1" ]; then
  echo "== pytest -m gpu" && timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  tail -2 "$OUT/pytest_gpu.log"
fi
echo "== bench" && timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
i=0
for v in ${VARIANTS:-}; do
  i=$((i+1))
  echo "== bench variant $v"
  timeout -k 10 600 python bench.py --no-cpu ${v//,/ } > "$OUT/bench_v$i.json" 2> "$OUT/bench_v$i.err"
  cat "$OUT/bench_v$i.json"
done
if [ "${PROF:-1}" = "1" ]; then
  echo "== rocprofv3"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e ${BENCH_ARGS:-} > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
fi
echo "== done"
