#!/bin/bash
# config 5b: one PMC pass (SQ instruction mix of k_long_dp) and rocprofv3 kernel stats
set -o pipefail
OUT=gpurun_out/${RUN:-r04w}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d $OUT/pmc -o run --output-format csv -- python3 bench.py --workload long-oov --steps 1 --warmup 1 --no-parity --no-e2e --no-profile \
  > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py --workload long-oov --steps 3 --warmup 1 --no-parity --no-e2e --no-profile \
  > $OUT/stats.log 2>&1 || { tail -5 $OUT/stats.log; exit 1; }
find $OUT -name "*counter_collection.csv" | head -2
find $OUT -name "*kernel_stats.csv" | head -2
