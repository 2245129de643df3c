# k_mark_walk: batched LDS reads in phase 1 and the hot-row lookups (ISA audit), A/B x3 + parity + phase clocks
set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "edge_cases or nonzh or zh_blocks_from_lane or config4 or random_mixed or record_overflow or golden or mini_dict" \
  > gpurun_out/r06e/pytest.log 2>&1 || exit 1
TAG=r06e REPS=3 STEPS=30 bash tools/abtest.sh base lib > gpurun_out/r06e/ab.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-e2e > gpurun_out/r06e/bench.json 2> gpurun_out/r06e/bench.err || exit 1
