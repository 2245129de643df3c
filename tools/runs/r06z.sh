# headline per-wave phase clocks (STAMPS build): k_zh and k_mark_walk, 1 GiB, HMM on
set -o pipefail
mkdir -p gpurun_out/r06z
JB_LIB=$PWD/jieba-go_amd/lib_st/libjiebahip.so JB_STAMPS=1 JB_GRAPH=0 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-e2e --no-parity --no-profile > gpurun_out/r06z/hl_stamps.json 2> gpurun_out/r06z/hl_stamps.err || exit 1
