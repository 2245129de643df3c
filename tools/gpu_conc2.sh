#!/bin/bash
# k_small coalescing: per-slot streams on their own CUs, by CU stride; JB_DEBUG batch logs
set -o pipefail
OUT=gpurun_out/${RUN:-conc2}; mkdir -p $OUT
for st in ${STRIDES:-1 32}; do
  echo "== JB_SMALL_CU_STRIDE=$st"
  JB_SMALL_CU_STRIDE=$st timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k concurrent -s \
    --timeout 150 --timeout-method thread > $OUT/pytest_s$st.log 2>&1 || { tail -20 $OUT/pytest_s$st.log; exit 1; }
  grep -E "JB_SMALL_SLOTS|serial threads|concurrent threads" $OUT/pytest_s$st.log
done
if [ -n "$DEBUG" ]; then
  JB_DEBUG=1 JB_CONC_LOG=$OUT/dbg timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k concurrent -s \
    --timeout 150 --timeout-method thread > $OUT/pytest_dbg.log 2>&1 || { tail -20 $OUT/pytest_dbg.log; exit 1; }
  python tools/conc_summary.py $OUT/dbg.slots*.txt
fi
