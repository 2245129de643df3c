# k_zh: the DP's block list in registers (RegSrc) + no claim when every group was a first; parity subset, A/B vs HEAD
set -o pipefail
mkdir -p gpurun_out/r06v
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "random_mixed or long_document or edge_cases or synthetic_golden or reference_kats or long_blocks_many" > gpurun_out/r06v/pytest.log 2>&1 || exit 1
for r in 1 2 3; do for v in base lib; do
  if [ $v = lib ]; then L=$PWD/jieba-go_amd/lib/libjiebahip.so; else L=$PWD/var/exp_$v/libjiebahip.so; fi
  JB_LIB=$L timeout -k 10 300 python -u bench.py --no-e2e --steps 20 --warmup 3 $( [ $r = 1 ] && [ $v = lib ] || echo --no-parity ) > gpurun_out/r06v/hl_${v}_$r.json 2> gpurun_out/r06v/hl_${v}_$r.err || exit 1
done; done
for r in 1 2; do for h in 0 1; do for v in base lib; do
  if [ $v = lib ]; then L=$PWD/jieba-go_amd/lib/libjiebahip.so; else L=$PWD/var/exp_$v/libjiebahip.so; fi
  JB_LIB=$L timeout -k 10 300 python -u bench.py --workload s10k --hmm $h --steps 300 --warmup 20 --no-e2e $( [ $r = 1 ] && [ $v = lib ] || echo --no-parity ) \
     > gpurun_out/r06v/s_h${h}_${v}_$r.json 2> gpurun_out/r06v/s_h${h}_${v}_$r.err || exit 1
done; done; done
