#!/bin/bash
# two walks per lane in k_mark_walk + k_long_dp register window: parity subset, A/B
set -o pipefail
OUT=gpurun_out/${RUN:-r04l}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "docs or golden or edge or overflow or long" \
  --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
TAG=${RUN:-r04l}/ablong bash tools/ab_long.sh lib ldrw1 ldold noring both || exit 1
TAG=${RUN:-r04l}/ab REPS=2 bash tools/abtest.sh lib mw1 || exit 1
