set -o pipefail
RUN=${RUN:-g1}
mkdir -p gpurun_out/$RUN
( nproc; python -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>&1; free -g | head -2 ) > gpurun_out/$RUN/env.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$RUN/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/$RUN/pytest.log; exit 1; }
tail -3 gpurun_out/$RUN/pytest.log
timeout -k 10 400 python -u bench.py > gpurun_out/$RUN/bench.json 2> gpurun_out/$RUN/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/$RUN/bench.err; exit 1; }
cat gpurun_out/$RUN/bench.json | head -c 3000
