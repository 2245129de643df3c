#!/bin/bash
# k_long_dp chain rewrite: long-block parity tests, config 5b bench; concurrency slots.
set -o pipefail
OUT=gpurun_out/${RUN:-r04k}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "long or edge or concurrent or docs or s10k or overflow or golden" -s --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -E "JB_SMALL_SLOTS|serial threads|concurrent threads" $OUT/pytest.log
timeout -k 10 300 python -u bench.py --workload long-oov --steps 5 --warmup 2 --no-e2e > $OUT/long_oov.json 2> $OUT/long_oov.err || { echo LONG_FAILED; tail -5 $OUT/long_oov.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/long_oov.json')); print('5b', d['ms_per_step'], d['kernels_ms']['k_long_dp'], d['parity']['bit_exact'])"
TAG=${RUN:-r04k}/ab REPS=2 bash tools/abtest.sh lib zhopt base
