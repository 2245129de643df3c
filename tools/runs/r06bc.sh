# k_zh: 256-block chunks (four per lane) at the default 6 KiB groups, weight table 4,608 entries (c256) vs HEAD (base)
set -o pipefail
O=gpurun_out/r06bc; mkdir -p $O
JB_LIB=$PWD/var/exp_c256/libjiebahip.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "synthetic_golden or random_mixed or long_document or zh_blocks or record_overflow or docs_corpus" > $O/pytest.log 2>&1 || exit 1
for r in 1 2 3; do for v in base c256; do
  JB_LIB=$PWD/var/exp_$v/libjiebahip.so timeout -k 10 300 python -u bench.py --no-e2e --no-latency --steps 20 --warmup 3 $( [ $r = 1 ] && [ $v = c256 ] || echo --no-parity ) > $O/hl_${v}_$r.json 2> $O/hl_${v}_$r.err || exit 1
done; done
for v in base c256; do
  JB_LIB=$PWD/var/exp_$v/libjiebahip.so timeout -k 10 300 python -u bench.py --no-e2e --no-latency --shard-of 8 --steps 20 --warmup 3 --no-parity > $O/s8_${v}.json 2> $O/s8_${v}.err || exit 1
done
