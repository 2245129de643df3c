# k_mark_walk split (two workgroups per tile for batches with at most one tile per CU): parity (auto and forced),
# S10k A/B x2 against HEAD, headline once each
set -o pipefail
O=gpurun_out/r06ac; mkdir -p $O
K="random_mixed or long_document or edge_cases or synthetic_golden or reference_kats or long_blocks_many or overflow or caller_arrays"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "$K" > $O/pytest_auto.log 2>&1 || exit 1
JB_MW_SPLIT=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "$K" > $O/pytest_forced.log 2>&1 || exit 1
lib() { if [ $1 = lib ]; then echo $PWD/jieba-go_amd/lib/libjiebahip.so; else echo $PWD/var/exp_$1/libjiebahip.so; fi; }
for r in 1 2; do for h in 0 1; do for v in base lib; do
  JB_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --workload s10k --hmm $h --steps 300 --warmup 20 --no-e2e $( [ $r = 1 ] && [ $v = lib ] || echo --no-parity ) \
     > $O/s_h${h}_${v}_$r.json 2> $O/s_h${h}_${v}_$r.err || exit 1
done; done; done
for v in base lib; do
  JB_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --no-e2e --steps 20 --warmup 3 --no-parity > $O/hl_${v}_1.json 2> $O/hl_${v}_1.err || exit 1
done
JB_MW_SPLIT=1 timeout -k 10 300 python -u bench.py --no-e2e --steps 5 --warmup 2 > $O/hl_forced.json 2> $O/hl_forced.err || exit 1
