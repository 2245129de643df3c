# 7 KiB k_zh groups in the wide form (384-byte slack, 256 blocks per chunk, 4,400 weights in LDS): parity with
# that build, then headline A/B x3 against HEAD and the default build of the parameterised source
set -o pipefail
O=gpurun_out/r06aq; mkdir -p $O
JB_LIB=$PWD/var/exp_g7/libjiebahip.so timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "random_mixed or long_document or edge_cases or synthetic_golden or reference_kats or overflow or repeat_runs or caller_arrays or long_blocks_many" > $O/pytest_g7.log 2>&1 || exit 1
lib() { if [ $1 = lib ]; then echo $PWD/jieba-go_amd/lib/libjiebahip.so; else echo $PWD/var/exp_$1/libjiebahip.so; fi; }
for r in 1 2 3; do for v in base lib g7; do
  JB_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --no-e2e --steps 20 --warmup 3 $( [ $r = 1 ] && [ $v = g7 ] || echo --no-parity ) > $O/hl_${v}_$r.json 2> $O/hl_${v}_$r.err || exit 1
done; done
