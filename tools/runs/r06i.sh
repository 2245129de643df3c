# S10k: k_zh narrow form with LDS weights (batched copy) vs gathered weights; parity first
set -o pipefail
mkdir -p gpurun_out/r06i
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  -k "edge_cases or nonzh or zh_blocks_from_lane or random_mixed or record_overflow or golden or mini_dict or docs_corpus or degenerate or s10k or small_batches or long_blocks_many or caller_log or add_word or graph_replay" \
  > gpurun_out/r06i/pytest.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in 0 1; do
    for h in 0 1; do
      JB_ZH_SMALL_LDS=$v timeout -k 10 300 python -u bench.py --workload s10k --hmm $h --steps 200 --warmup 20 --no-e2e --no-parity \
        > gpurun_out/r06i/s10k_h${h}_lds${v}_$rep.json 2> gpurun_out/r06i/s10k_h${h}_lds${v}_$rep.err || exit 1
    done
  done
done
timeout -k 10 300 python -u bench.py --workload s10k --hmm 1 --no-e2e > gpurun_out/r06i/s10k_h1_parity.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py --workload s10k --hmm 0 --no-e2e > gpurun_out/r06i/s10k_h0_parity.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06i/s10k_h0 -o s10k -- python3 $GRAFT_REPO_ROOT/bench.py --workload s10k --hmm 0 --steps 200 --warmup 20 --no-e2e --no-parity --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r06i/s10k_h0.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06i/s10k_h0.err || exit 1
