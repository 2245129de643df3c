# usage: bash tools/runs/abrun.sh TAG  — GPU parity subset, then headline A/B x3 (base vs lib) and S10k
# HMM off/on A/B x2; the first lib run of each workload checks parity against the oracle.
set -o pipefail
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "${PYK:-random_mixed or long_document or edge_cases or synthetic_golden or reference_kats or long_blocks_many}" > $O/pytest.log 2>&1 || exit 1
lib() { if [ $1 = lib ]; then echo $PWD/jieba-go_amd/lib/libjiebahip.so; else echo $PWD/var/exp_$1/libjiebahip.so; fi; }
for r in $(seq 1 ${HLREPS:-3}); do for v in ${VARIANTS:-base lib}; do
  JB_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --no-e2e --steps 20 --warmup 3 $( [ $r = 1 ] && [ $v = lib ] || echo --no-parity ) > $O/hl_${v}_$r.json 2> $O/hl_${v}_$r.err || exit 1
done; done
for r in $(seq 1 ${SREPS:-2}); do for h in 0 1; do for v in ${VARIANTS:-base lib}; do
  JB_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --workload s10k --hmm $h --steps 300 --warmup 20 --no-e2e $( [ $r = 1 ] && [ $v = lib ] || echo --no-parity ) \
     > $O/s_h${h}_${v}_$r.json 2> $O/s_h${h}_${v}_$r.err || exit 1
done; done; done
