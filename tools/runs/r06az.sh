# k_nonzh occupancy variants vs HEAD (base): nzA = 64-chunk rounds (one per lane), nzF = nonzh_block's
# per-byte path out of line, nzG = both; every variant parity-checked on the 1 GiB
O=gpurun_out/r06az; mkdir -p $O
for r in 1 2; do for v in base nzA nzF nzG; do
  JB_LIB=$PWD/var/exp_$v/libjiebahip.so timeout -k 10 300 python -u bench.py --no-e2e $( [ $r = 1 ] && [ $v != base ] || echo --no-parity ) --steps 20 --warmup 3 > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 1
done; done
