#!/bin/bash
# k_long_dp positional-descriptor chain: parity subset, chain microbenchmark, 5b A/B
set -o pipefail
OUT=gpurun_out/${RUN:-r04m}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "long or edge or golden or overflow" \
  --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
true
true
TAG=${RUN:-r04m}/ablong REPS=2 bash tools/ab_long.sh lib uni rw2 || exit 1
