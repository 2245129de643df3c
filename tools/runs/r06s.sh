# S10k: k_zh wide (weights in LDS) vs narrow form, stamps build (per-wave DP clocks) and the timed build
set -o pipefail
mkdir -p gpurun_out/r06s
for w in 0 1; do
  JB_ZH_WIDE=$w JB_LIB=$PWD/jieba-go_amd/lib_st/libjiebahip.so JB_STAMPS=1 JB_GRAPH=0 timeout -k 10 300 python -u bench.py --workload s10k --hmm 0 --steps 3 --warmup 1 --no-e2e --no-parity --no-profile \
     > gpurun_out/r06s/st_w$w.json 2> gpurun_out/r06s/st_w$w.err || exit 1
  JB_ZH_WIDE=$w timeout -k 10 300 python -u bench.py --workload s10k --hmm 0 --steps 200 --warmup 20 --no-e2e --no-parity \
     > gpurun_out/r06s/t_w$w.json 2> gpurun_out/r06s/t_w$w.err || exit 1
done
