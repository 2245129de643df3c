#!/bin/bash
# decided chain on 5b: STAMPS clocks (chain vs helpers, fallback count)
set -o pipefail
OUT=gpurun_out/${RUN:-r04y}; mkdir -p $OUT
JB_LIB=$PWD/jieba-go_amd/lib_st/libjiebahip.so JB_STAMPS=1 JB_GRAPH=0 timeout -k 10 300 \
  python -u bench.py --workload long-oov --steps 1 --warmup 1 --no-parity --no-e2e --no-profile > $OUT/st_long.json 2> $OUT/st_long.err \
  || { tail -5 $OUT/st_long.err; exit 1; }
grep "k_long_dp wg" $OUT/st_long.err | head -3
