# k_tok write pass: LDS staging capacity 2304 / 2560 tokens per tile (less LDS, more workgroups per CU) vs HEAD's 3072 (base)
O=gpurun_out/r06be; mkdir -p $O
for r in 1 2 3; do for v in base tc2304 tc2560; do
  JB_LIB=$PWD/var/exp_$v/libjiebahip.so timeout -k 10 300 python -u bench.py --no-e2e --no-latency --steps 20 --warmup 3 $( [ $r = 1 ] && [ $v != base ] || echo --no-parity ) > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 1
done; done
