# k_nonzh timing ablations at 1 GiB (wrong tokens): no docbits clearing, block end = chunk end, no tokenizing
set -o pipefail
O=gpurun_out/r06as; mkdir -p $O
for v in base nzdocs nzend nzblock base; do
  L=$PWD/var/exp_$v/libjiebahip.so
  JB_LIB=$L timeout -k 10 300 python -u bench.py --no-e2e --no-parity --steps 20 --warmup 3 > $O/$v.json 2>> $O/$v.err || exit 1
done
