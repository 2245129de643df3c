# S10k: the window's records pulled into the caches before the DP (JB_ZH_TOUCH) A/B, stamps + timed
set -o pipefail
mkdir -p gpurun_out/r06t
for t in 0 1; do
  JB_ZH_TOUCH=$t JB_LIB=$PWD/jieba-go_amd/lib_st/libjiebahip.so JB_STAMPS=1 JB_GRAPH=0 timeout -k 10 300 python -u bench.py --workload s10k --hmm 0 --steps 3 --warmup 1 --no-e2e --no-parity --no-profile \
     > gpurun_out/r06t/st_t$t.json 2> gpurun_out/r06t/st_t$t.err || exit 1
done
for r in 1 2; do for h in 0 1; do for t in 0 1; do
  JB_ZH_TOUCH=$t timeout -k 10 300 python -u bench.py --workload s10k --hmm $h --steps 200 --warmup 20 --no-e2e $( [ $r = 1 ] || echo --no-parity ) \
     > gpurun_out/r06t/t_h${h}_t${t}_$r.json 2> gpurun_out/r06t/t_h${h}_t${t}_$r.err || exit 1
done; done; done
