set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 180 --timeout-method thread -k "long_wait_bound or long_blocks_many or edge_cases or concurrent_cut_calls" > gpurun_out/r06a/pytest.log 2>&1 && \
for n in 2 4 8; do timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --shard-of $n --no-e2e --no-latency > gpurun_out/r06a/shard$n.json 2> gpurun_out/r06a/shard$n.err || exit 1; done
