#!/bin/bash
# Round 4: diagnostics after k_zh's wide form: k_long_dp chain clocks (STAMPS, config 5b),
# the concurrent Cut program's rates, headline STAMPS clocks, PMC passes.
set -o pipefail
OUT=gpurun_out/${RUN:-r04f}
mkdir -p $OUT
export TMPDIR=/tmp
JB_LIB=$PWD/jieba-go_amd/lib_st/libjiebahip.so JB_STAMPS=1 JB_GRAPH=0 timeout -k 10 200 python -u bench.py --workload long-oov --steps 1 --warmup 1 --no-parity --no-e2e --no-profile > $OUT/st_long.json 2> $OUT/st_long.err || { echo ST_LONG_FAILED; tail -5 $OUT/st_long.err; exit 1; }
grep "k_long_dp wg" $OUT/st_long.err | head -3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k concurrent -s --timeout 250 --timeout-method thread > $OUT/concurrent.log 2>&1 || { echo CONC_FAILED; tail -20 $OUT/concurrent.log; exit 1; }
grep -E "^serial|^concurrent" $OUT/concurrent.log
JB_LIB=$PWD/jieba-go_amd/lib_st/libjiebahip.so JB_STAMPS=1 JB_GRAPH=0 timeout -k 10 200 python -u bench.py --corpus-mib 256 --steps 1 --warmup 1 --no-parity --no-e2e --no-profile --no-latency > $OUT/st_docs.json 2> $OUT/st_docs.err || { echo ST_DOCS_FAILED; tail -5 $OUT/st_docs.err; exit 1; }
grep "clocks" $OUT/st_docs.err | tail -2
TAG=${RUN:-r04f}/pmc bash tools/pmc.sh > $OUT/pmc.log 2>&1 || { echo PMC_FAILED; tail -5 $OUT/pmc.log; exit 1; }
python3 tools/pmc_summary.py $OUT/pmc $OUT/pmc_latest.json "1 GiB C_syn corpus, prefix dict, hmm on; r04f" > $OUT/pmc_summary.txt 2>&1
tail -30 $OUT/pmc_summary.txt
