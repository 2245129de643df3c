# S10k's k_zh and k_mark_walk per-wave phase clocks (STAMPS build), HMM off and on
set -o pipefail
mkdir -p gpurun_out/r06r
for h in 0 1; do
  JB_LIB=$PWD/jieba-go_amd/lib_st/libjiebahip.so JB_STAMPS=1 JB_GRAPH=0 timeout -k 10 300 python -u bench.py --workload s10k --hmm $h --steps 3 --warmup 1 --no-e2e --no-parity --no-profile \
     > gpurun_out/r06r/s10k_h$h.json 2> gpurun_out/r06r/s10k_h$h.err || exit 1
done
