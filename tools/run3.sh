set -o pipefail
RUN=${RUN:-r03b}
mkdir -p gpurun_out/$RUN
JB_LIB=var/g12/libjiebahip.so JB_TEST_ZH_GROUPS=12288 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k zh_groups --timeout 200 --timeout-method thread > gpurun_out/$RUN/pytest_g12.log 2>&1 || { echo PYTEST_G12_FAILED; tail -30 gpurun_out/$RUN/pytest_g12.log; exit 1; }
tail -1 gpurun_out/$RUN/pytest_g12.log
timeout -k 10 400 python -u bench.py > gpurun_out/$RUN/bench.json 2> gpurun_out/$RUN/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/$RUN/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/$RUN/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['parity']['bit_exact'], json.dumps(d['end_to_end_host']))"
