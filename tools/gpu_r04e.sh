#!/bin/bash
# Round 4: GPU suite, A/B of k_zh's wide form (JB_ZH_WIDE=0 vs default), config 5b.
set -o pipefail
OUT=gpurun_out/${RUN:-r04e}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
grep -A3 "concurrent_cut_calls" $OUT/pytest.log | grep -E "serial|concurrent" | head -4
TAG=${RUN:-r04e}/ab REPS=2 bash tools/envab.sh JB_ZH_WIDE=0 - || exit 1
timeout -k 10 300 python -u bench.py --workload long-oov --steps 5 --warmup 2 --no-e2e > $OUT/long_oov.json 2> $OUT/long_oov.err || { echo LONG_FAILED; tail -5 $OUT/long_oov.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/long_oov.json')); print('5b', d['ms_per_step'], d['kernels_ms'], d['parity']['bit_exact'])"
