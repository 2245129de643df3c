#!/bin/bash
# GPU suite on the in-tree library, then A/B against var/exp_<V...> variants.
# usage: RUN=r04g VARS="base" bash tools/gpu_ab.sh
set -o pipefail
OUT=gpurun_out/${RUN:-ab}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
TAG=${RUN:-ab}/ab REPS=${REPS:-2} bash tools/abtest.sh lib ${VARS:-base}
