#!/bin/bash
# One GPU call: the -m gpu suite, the 12 KiB k_zh group build on its group test
# (if built: make -C jieba-go_amd ZH_GROUP=12288 OUT=../var/g12 OBJ=../var/g12o), then
# the default bench line.  usage: RUN=r03a bash tools/gpu_check.sh
set -o pipefail
RUN=${RUN:-g1}
mkdir -p gpurun_out/$RUN
( nproc; python -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>&1; free -g | head -2 ) > gpurun_out/$RUN/env.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/$RUN/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/$RUN/pytest.log; exit 1; }
tail -3 gpurun_out/$RUN/pytest.log
if [ -f var/g12/libjiebahip.so ]; then
  JB_LIB=var/g12/libjiebahip.so JB_TEST_ZH_GROUPS=12288 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k zh_groups --timeout 200 --timeout-method thread > gpurun_out/$RUN/pytest_g12.log 2>&1 || { echo PYTEST_G12_FAILED; tail -30 gpurun_out/$RUN/pytest_g12.log; exit 1; }
  tail -2 gpurun_out/$RUN/pytest_g12.log
fi
timeout -k 10 400 python -u bench.py > gpurun_out/$RUN/bench.json 2> gpurun_out/$RUN/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/$RUN/bench.err; exit 1; }
cat gpurun_out/$RUN/bench.json | head -c 3000
