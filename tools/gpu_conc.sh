#!/bin/bash
set -o pipefail
OUT=gpurun_out/${RUN:-conc}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k concurrent -s --timeout 250 --timeout-method thread > $OUT/concurrent.log 2>&1 || { echo CONC_FAILED; tail -20 $OUT/concurrent.log; exit 1; }
grep -E "JB_SMALL_SLOTS|serial|concurrent threads" $OUT/concurrent.log
