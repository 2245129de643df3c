# Long-block (k_long_*) checks on the GPU box: focused parity tests, then the
# config-5 benches (bit-exact against the oracle inside bench.py).
set -o pipefail
RUN=${RUN:-l1}
mkdir -p gpurun_out/$RUN
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "${TESTS:-long or edge or ties or overflow or golden}" > gpurun_out/$RUN/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/$RUN/pytest.log; exit 1; }
tail -3 gpurun_out/$RUN/pytest.log
for w in long-oov long-punct; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 1 --no-e2e > gpurun_out/$RUN/$w.json 2> gpurun_out/$RUN/$w.err || { echo BENCH_FAILED $w; tail -20 gpurun_out/$RUN/$w.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/$RUN/$w.json')); print('$w', d['ms_per_step'], d['kernels_ms'], d['parity'], d['cpu_baseline']['value'])"
done
