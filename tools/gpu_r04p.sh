#!/bin/bash
# k_long_dp: parity subset, 5b A/B, per-window chain clocks (STAMPS build) fitted by group kind
set -o pipefail
OUT=gpurun_out/${RUN:-r04p}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "long or edge or golden or overflow" \
  --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
JB_LIB=$PWD/jieba-go_amd/lib_st/libjiebahip.so JB_STAMPS=1 JB_GRAPH=0 JB_LDW_OUT=$OUT/ldw.bin timeout -k 10 200 \
  python -u bench.py --workload long-oov --steps 1 --warmup 1 --no-parity --no-e2e --no-profile > $OUT/st_long.json 2> $OUT/st_long.err \
  || { tail -5 $OUT/st_long.err; exit 1; }
grep "k_long_dp wg" $OUT/st_long.err | head -2
python tools/ldw_fit.py $OUT/ldw.bin
TAG=${RUN:-r04p}/ablong REPS=2 bash tools/ab_long.sh ${VARS:-lib rw2} || exit 1
