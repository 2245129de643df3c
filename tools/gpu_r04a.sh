#!/bin/bash
# Round 4 first GPU call: -m gpu suite, the default bench line, and bench.py --gpus 2
# on the 1-GPU box (must refuse).  usage: RUN=r04a bash tools/gpu_r04a.sh
set -o pipefail
RUN=${RUN:-r04a}
mkdir -p gpurun_out/$RUN
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/$RUN/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/$RUN/pytest.log; exit 1; }
tail -3 gpurun_out/$RUN/pytest.log
timeout -k 10 400 python -u bench.py > gpurun_out/$RUN/bench.json 2> gpurun_out/$RUN/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/$RUN/bench.err; exit 1; }
head -c 1500 gpurun_out/$RUN/bench.json
timeout -k 10 120 python -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/$RUN/bench2.json 2> gpurun_out/$RUN/bench2.err
echo "gpus2 rc=$? (want non-zero)"; cat gpurun_out/$RUN/bench2.err | tail -3
