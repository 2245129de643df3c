# k_mark_walk: run links and level 1 per lane from registers; parity, A/B x3 against the two builds before
set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "edge_cases or nonzh or zh_blocks_from_lane or config4 or random_mixed or record_overflow or golden or mini_dict or long_document or docs_corpus or degenerate or s10k or small_batches" \
  > gpurun_out/r06f/pytest.log 2>&1 || exit 1
TAG=r06f REPS=3 STEPS=30 bash tools/abtest.sh base lds lib > gpurun_out/r06f/ab.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-e2e > gpurun_out/r06f/bench.json 2> gpurun_out/r06f/bench.err || exit 1
