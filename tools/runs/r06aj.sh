# headline DP balance stamps (longest block per chunk), and the new determinism test + parity subset on this build
set -o pipefail
O=gpurun_out/r06aj; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "repeat_runs or random_mixed or caller_arrays or overflow or edge_cases" > $O/pytest.log 2>&1 || exit 1
JB_LIB=$PWD/jieba-go_amd/lib_st/libjiebahip.so JB_STAMPS=1 JB_GRAPH=0 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-e2e --no-parity --no-profile > $O/hl_stamps.json 2> $O/hl_stamps.err || exit 1
