#!/bin/bash
# round-end evidence on the decided chain: full GPU suite, smoke + headline + configs + sentence
# stats (tools/round_end.sh), then 5b PMC + rocprofv3 stats (tools/gpu_r04w.sh)
set -o pipefail
T=${TAG:-r04z}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
TAG=$T bash tools/round_end.sh || exit 1
RUN=$T/w bash tools/gpu_r04w.sh || exit 1
echo done
