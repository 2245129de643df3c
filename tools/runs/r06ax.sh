# k_nonzh floor ablations on r06av: nz1 = alnum16 + wave scan only, nz2 = + chunk list and loads, nz3 = half the workgroups (2 units per wave)
# nz2 = + block end clipped to the chunk, nz3 = + no walk-back; lib = mask fast path
O=gpurun_out/r06ax; mkdir -p $O
for v in lib nz1 nz2 nz3 lib; do
  L=$PWD/var/exp_$v/libjiebahip.so; [ $v = lib ] && L=$PWD/jieba-go_amd/lib/libjiebahip.so
  JB_LIB=$L timeout -k 10 300 python -u bench.py --no-e2e --no-parity --steps 20 --warmup 3 > $O/$v.json 2> $O/$v.err || exit 1
done
