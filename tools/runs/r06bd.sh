# timing ablation (wrong tokens): Emitter flushes as plain stores instead of atomicOr (nzst) vs HEAD (base)
O=gpurun_out/r06bd; mkdir -p $O
for r in 1 2; do for v in base nzst; do
  JB_LIB=$PWD/var/exp_$v/libjiebahip.so timeout -k 10 300 python -u bench.py --no-e2e --no-latency --no-parity --steps 20 --warmup 3 > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 1
done; done
