# k_tok1's tiles as k_long's last phase (small batches): full GPU suite, then S10k A/B x3 against HEAD
set -o pipefail
O=gpurun_out/r06al; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1 || exit 1
JB_TOK_FUSE=0 timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "random_mixed or long_blocks_many or repeat_runs" > $O/pytest_nofuse.log 2>&1 || exit 1
lib() { if [ $1 = lib ]; then echo $PWD/jieba-go_amd/lib/libjiebahip.so; else echo $PWD/var/exp_$1/libjiebahip.so; fi; }
for r in 1 2 3; do for h in 0 1; do for v in base lib; do
  JB_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --workload s10k --hmm $h --steps 300 --warmup 20 --no-e2e $( [ $r = 1 ] && [ $v = lib ] || echo --no-parity ) \
     > $O/s_h${h}_${v}_$r.json 2> $O/s_h${h}_${v}_$r.err || exit 1
done; done; done
for v in base lib; do
  JB_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --workload long-punct --steps 20 --warmup 3 --no-e2e $( [ $v = lib ] || echo --no-parity ) > $O/l1m_${v}.json 2> $O/l1m_${v}.err || exit 1
done
