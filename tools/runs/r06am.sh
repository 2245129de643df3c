# S10k DP timing ablations (STAMPS builds, wrong tokens): base, weights from 16 entries (ablw), no ring reads (ablr)
set -o pipefail
O=gpurun_out/r06am; mkdir -p $O
for v in base ablw ablr base; do
  if [ $v = base ]; then L=$PWD/jieba-go_amd/lib_st/libjiebahip.so; else L=$PWD/var/exp_$v/libjiebahip.so; fi
  JB_LIB=$L JB_STAMPS=1 JB_GRAPH=0 timeout -k 10 300 python -u bench.py --workload s10k --hmm 0 --steps 3 --warmup 1 --no-e2e --no-parity --no-profile > $O/$v.json 2>> $O/$v.err || exit 1
done
