# k_mark_walk split 2^s, s = 1/2/3 on S10k (same build), parity with s = 2 and 3 forced
set -o pipefail
O=gpurun_out/r06ad; mkdir -p $O
K="random_mixed or long_document or edge_cases or synthetic_golden or reference_kats or overflow or caller_arrays"
for m in 2 3; do
JB_MW_SPLIT=$m timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "$K" > $O/pytest_s$m.log 2>&1 || exit 1
done
for r in 1 2; do for h in 0 1; do for m in 1 2 3; do
  JB_MW_SPLIT=$m timeout -k 10 300 python -u bench.py --workload s10k --hmm $h --steps 300 --warmup 20 --no-e2e $( [ $r = 1 ] || echo --no-parity ) \
     > $O/s_h${h}_s${m}_$r.json 2> $O/s_h${h}_s${m}_$r.err || exit 1
done; done; done
